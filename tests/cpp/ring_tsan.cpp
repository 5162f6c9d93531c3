// ring_tsan.cpp -- the ShMemSymBuff reader/writer protocol under
// ThreadSanitizer (host only).  ring_test.cpp runs writer and reader as two
// processes, which TSan cannot follow (two mappings of one segment); here one
// ring object is shared by a writer thread and a reader thread, so every
// access to the slots and the ring indices is seen at one address and the
// acquire/release ordering of the protocol is checked.
// Build: g++ -O1 -g -fsanitize=thread -std=c++17 -I<pkg>/host -DnumOfRows=2
//        -Ddimension=16 -Dprefix=P -DlenOfBuffer=L -DshmemID='"/name"'
// Usage: ring_tsan <nsymbols> <wait|nowait>   (exit 0 on success)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "ShMemSymBuff.hpp"

static const int kRow = dimension + prefix;

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 3 * lenOfBuffer;
    const bool wait = argc > 2 ? strcmp(argv[2], "nowait") != 0 : true;
    ShMemSymBuff ring(shmemID, 1);
    std::thread writer([&] {
        std::vector<complexF> sym((size_t)numOfRows * kRow);
        for (int i = 0; i < n; ++i) {
            for (int r = 0; r < numOfRows; ++r)
                for (int k = 0; k < kRow; ++k)
                    sym[(size_t)r * kRow + k] = complexF{(float)(i * 1000 + r * 100 + (k - prefix)), (float)-i};
            if (wait) {
                ring.writeNextSymbolWithWait(sym.data());
            } else {
                ring.writeNextSymbolNoWait(sym.data());
                std::this_thread::sleep_for(std::chrono::milliseconds(3));
            }
        }
    });
    std::vector<complexF> y((size_t)numOfRows * dimension);
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        if (i == n - 1)
            ring.readLastSymbol(y.data());
        else
            ring.readNextSymbol(y.data(), i % lenOfBuffer);
        for (int r = 0; r < numOfRows; ++r)
            for (int k = 0; k < dimension; ++k) {
                const complexF v = y[(size_t)r * dimension + k];
                if (v.real != (float)(i * 1000 + r * 100 + k) || v.imag != (float)-i) ++bad;
            }
    }
    writer.join();
    std::printf("%s: %d symbols, %d bad samples\n", bad ? "FAIL" : "ok", n, bad);
    return bad ? 1 : 0;
}
