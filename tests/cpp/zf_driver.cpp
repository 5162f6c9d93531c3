// zf_driver.cpp -- the reference's zero-forcing call sequence
// (createZeroForcingMatrix then multiplyWithChannelInv, cpuLS.hpp:415-463)
// written against this package's cpuLS.hpp.
//   zf_driver rows cols users   reads  H.bin (users x rows x (cols-1) cube),
//                                      X.bin (users x (cols-1) symbol)
//                               writes W.bin (the H output), Xrot.bin (the
//                                      cube after the in-place rotCube),
//                                      HX.bin (rows x (cols-1))
#include <cstdio>
#include <vector>

#include "cpuLS.hpp"

static std::vector<complexF> load(const char *path, size_t n) {
    std::vector<complexF> v(n);
    FILE *f = std::fopen(path, "rb");
    if (!f || std::fread(v.data(), sizeof(complexF), n, f) != n) {
        std::fprintf(stderr, "cannot read %s\n", path);
        std::exit(2);
    }
    std::fclose(f);
    return v;
}
static void store(const char *path, const std::vector<complexF> &v) {
    FILE *f = std::fopen(path, "wb");
    std::fwrite(v.data(), sizeof(complexF), v.size(), f);
    std::fclose(f);
}

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    const int rows = std::atoi(argv[1]), cols = std::atoi(argv[2]), users = std::atoi(argv[3]);
    const size_t K = cols - 1;
    std::vector<complexF> X = load("H.bin", (size_t)users * rows * K);
    std::vector<complexF> sym = load("X.bin", (size_t)users * K);
    std::vector<complexF> H((size_t)users * rows * K), HX((size_t)rows * K);
    createZeroForcingMatrix(H.data(), X.data(), rows, cols, users);
    multiplyWithChannelInv(HX.data(), sym.data(), H.data(), rows, cols, users);
    store("W.bin", H);
    store("Xrot.bin", X);
    store("HX.bin", HX);
    return 0;
}
