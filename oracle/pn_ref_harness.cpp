// pn_ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (oracle/build_ref.sh).
//
// extern "C" entry around the reference's own PN correlator: build_ref.sh
// replaces the marker line below with rx_and_corr.cpp's correlator block
// (the `temp` declaration through the end of `if (corr_flag == false)`,
// rx_and_corr.cpp:329-360), read where it lies in /root/reference -- the
// UHD/boost radio loop around it cannot be built here.  The variables the
// block uses are declared with the reference's own types
// (rx_and_corr.cpp:97, 147, 233, 265, 299-300).  One call searches the
// channels of `buf` in the reference's order and returns the first hit's lag
// (`length`), or -1; *mag receives the block's last temp_iter (the hit's
// |corr|/L when there is one).  The block's std::cout report of a hit is
// discarded.
#include <cmath>
#include <complex>
#include <iostream>
#include <sstream>
#include <vector>

extern "C" long long ref_pn_correlate(const float *buf_f, int R, int N, const float *pn_f, int L,
                                      float thres, float *mag) {
    const auto *b = reinterpret_cast<const std::complex<float> *>(buf_f);
    const auto *p = reinterpret_cast<const std::complex<float> *>(pn_f);
    std::vector<size_t> channel_nums(R);
    std::vector<std::complex<float> > pn_buff(p, p + L);
    std::vector<std::vector<std::complex<float> > > buff1(R);
    for (int ch = 0; ch < R; ch++) buff1[ch].assign(b + (size_t)ch * N, b + (size_t)(ch + 1) * N);
    int samps_per_buff = N, length = 0;
    bool corr_flag = false;
    size_t num_rx_samps = N;
    std::ostringstream sink;
    std::streambuf *keep = std::cout.rdbuf(sink.rdbuf());
    // @@REFERENCE_CORRELATOR_BLOCK@@
    std::cout.rdbuf(keep);
    *mag = temp_iter;
    return corr_flag ? length : -1;
}
