// rx_writer_harness.cpp -- TEST INFRASTRUCTURE ONLY (oracle/build_drivers.sh).
//
// main() for the reference's own ring-writer code: build_drivers.sh feeds
// g++ rx_and_corr.cpp's include/configuration block (rx_and_corr.cpp:48-61:
// #include "ShMemSymBuff_gpu.hpp", mode, buffPtr, the SIGINT flag,
// copy_buff, cp_size) and its copy_to_shared_mem (rx_and_corr.cpp:64-87)
// unchanged, straight from /root/reference, in front of this file; the
// UHD/boost radio loop around them cannot be built here.  This main plays the
// part of that loop (rx_and_corr.cpp:296-305, 366-399): copy_buff holds
// numOfRows channels of numSymbols*(FFT_size+cp_size) samples read from a
// file (channel-major), the ring is opened as master, and -- as the radio
// loop hands over one synchronised frame per buffer pair until SIGINT -- the
// same frame is pushed with copy_to_shared_mem(numOfRows) (numSymbols
// writeNextSymbolNoWait calls, cyclic prefix dropped) every 50 ms until
// SIGINT or until the reader detaches.  The repetition matters: the NoWait
// writer never waits for the reader, so a reader that attaches late (a GPU
// driver initialising HIP) catches a later frame, exactly as it would behind
// the radio.  usage: rx_writer <iq file> <cp_size>
#include <chrono>
#include <csignal>
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
    std::signal(SIGINT, &sig_int_handler);
    buffPtr = new ShMemSymBuff(shmemID, mode);
    CSharedMemSimple view(shmemID, sizeof(symbolBuffer));
    auto *sb = static_cast<symbolBuffer *>(view.ptr());
    int frames = 0;
    for (; frames < 2400 && !stop_signal_called && __atomic_load_n(&sb->size, __ATOMIC_ACQUIRE) != -1; ++frames) {
        copy_to_shared_mem(numOfRows);
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    std::printf("rx_writer: %d frames of %d symbols\n", frames, numSymbols);
    delete buffPtr;
    return 0;
}
