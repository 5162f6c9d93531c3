// ring_test.cpp -- two processes over the ShMemSymBuff ring (host only).
// Build: g++ -O2 -std=c++17 -I<pkg>/host -DnumOfRows=2 -Ddimension=16
//        -Dprefix=P -DlenOfBuffer=L -DshmemID='"/name"' ring_test.cpp
// Usage: ring_test <nsymbols> <writer: wait|nowait>
// The child is the master/writer, the parent the slave/reader.  Symbol i
// carries sample values (i*1000 + k, -i); the reader checks order and
// content (prefix dropped).  Exit 0 on success.
#include <sys/wait.h>
#include <unistd.h>

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
    pid_t pid = fork();
    if (pid == 0) {  // writer / master
        ShMemSymBuff ring(shmemID, 1);
        std::vector<complexF> sym((size_t)numOfRows * kRow);
        for (int i = 0; i < n; ++i) {
            for (int r = 0; r < numOfRows; ++r)
                for (int k = 0; k < kRow; ++k)
                    sym[(size_t)r * kRow + k] =
                        complexF{(float)(i * 1000 + r * 100 + (k - prefix)), (float)-i};
            if (wait) {
                ring.writeNextSymbolWithWait(sym.data());
            } else {
                ring.writeNextSymbolNoWait(sym.data());
                std::this_thread::sleep_for(std::chrono::milliseconds(2));
            }
        }
        // keep the segment alive until the reader is done (bounded)
        for (int t = 0; t < 5000; ++t) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        _exit(0);
    }
    ShMemSymBuff ring(shmemID, 0);
    std::vector<complexF> Y((size_t)numOfRows * dimension);
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        if (i == n - 1)
            ring.readLastSymbol(Y.data());
        else
            ring.readNextSymbol(Y.data(), i % numberOfSymbolsToTest);
        for (int r = 0; r < numOfRows; ++r)
            for (int k = 0; k < dimension; ++k) {
                const complexF v = Y[(size_t)r * dimension + k];
                if (v.real != (float)(i * 1000 + r * 100 + k) || v.imag != (float)-i) ++bad;
            }
        if (bad) {
            fprintf(stderr, "symbol %d: %d bad samples (got %g,%g)\n", i, bad, Y[0].real, Y[0].imag);
            break;
        }
    }
    int status = 0;
    kill(pid, SIGTERM);
    waitpid(pid, &status, 0);
    printf("ring_test: %d symbols, %s\n", n, bad ? "FAIL" : "ok");
    return bad ? 1 : 0;
}
