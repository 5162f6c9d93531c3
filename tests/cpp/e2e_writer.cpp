// e2e_writer.cpp -- master/writer side of the end-to-end test: pushes the
// symbols of a raw IQ file (nsym x numOfRows x (dimension+prefix) complex
// floats) into the ShMemSymBuff ring, like rx_and_corr.cpp's
// copy_to_shared_mem (rx_and_corr.cpp:64-87), then waits (bounded) for the
// reader to detach.  usage: e2e_writer <iq file> [repeat]: the file's symbols
// are pushed `repeat` times (a long synthetic stream for the ingest rate).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <thread>
#include <vector>

#include "ShMemSymBuff.hpp"

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    std::ifstream f(argv[1], std::ifstream::binary | std::ifstream::ate);
    const size_t per = (size_t)numOfRows * (dimension + prefix);
    const size_t nsym = (size_t)f.tellg() / (per * sizeof(complexF));
    f.seekg(0);
    const int repeat = argc > 2 ? std::atoi(argv[2]) : 1;
    std::vector<complexF> all(per * nsym);
    f.read(reinterpret_cast<char *>(all.data()), (std::streamsize)(all.size() * sizeof(complexF)));
    ShMemSymBuff ring(shmemID, 1);
    for (int k = 0; k < repeat; ++k)
        for (size_t i = 0; i < nsym; ++i) ring.writeNextSymbolWithWait(&all[i * per]);
    // hold the segment until the slave detaches (size = -1), at most 120 s
    CSharedMemSimple view(shmemID, sizeof(symbolBuffer));
    auto *sb = static_cast<symbolBuffer *>(view.ptr());
    for (int t = 0; t < 120000 && __atomic_load_n(&sb->size, __ATOMIC_ACQUIRE) != -1; ++t)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    std::printf("writer: %zu symbols\n", nsym * repeat);
    return 0;
}
