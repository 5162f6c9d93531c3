// rx_writer_harness.cpp -- TEST INFRASTRUCTURE ONLY (oracle/build_drivers.sh).
//
// main() for the reference's own ring-writer code: build_drivers.sh feeds
// g++ rx_and_corr.cpp's include/configuration block (rx_and_corr.cpp:48-60:
// #include "ShMemSymBuff_gpu.hpp", mode, buffPtr, copy_buff, cp_size) and its
// copy_to_shared_mem (rx_and_corr.cpp:64-87) unchanged, straight from
// /root/reference, in front of this file; the UHD/boost radio loop around
// them cannot be built here.  This main plays the part of that loop after
// frame sync (rx_and_corr.cpp:298-302, 366-399): it fills copy_buff with
// numOfRows channels of numSymbols*(FFT_size+cp_size) samples read from a
// file (channel-major), opens the ring as master, calls
// copy_to_shared_mem(numOfRows) -- numSymbols writeNextSymbolNoWait calls
// with the cyclic prefix dropped -- and waits (bounded) for the reader to
// detach.  usage: rx_writer <iq file> <cp_size>
#include <chrono>
#include <thread>

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    cp_size = std::atoi(argv[2]);
    const size_t per_ch = (size_t)numSymbols * (FFT_size + cp_size);
    std::ifstream f(argv[1], std::ifstream::binary);
    copy_buff.assign(numOfRows, std::vector<std::complex<float>>(per_ch));
    for (int ch = 0; ch < numOfRows; ++ch)
        f.read(reinterpret_cast<char *>(copy_buff[ch].data()),
               (std::streamsize)(per_ch * sizeof(std::complex<float>)));
    if (!f) {
        std::fprintf(stderr, "rx_writer: short input file\n");
        return 1;
    }
    buffPtr = new ShMemSymBuff(shmemID, mode);
    copy_to_shared_mem(numOfRows);
    CSharedMemSimple view(shmemID, sizeof(symbolBuffer));
    auto *sb = static_cast<symbolBuffer *>(view.ptr());
    for (int t = 0; t < 120000 && __atomic_load_n(&sb->size, __ATOMIC_ACQUIRE) != -1; ++t)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    std::printf("rx_writer: %d symbols\n", numSymbols);
    delete buffPtr;
    return 0;
}
