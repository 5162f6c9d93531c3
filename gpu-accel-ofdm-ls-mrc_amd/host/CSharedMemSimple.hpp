// CSharedMemSimple.hpp -- POSIX shared-memory segment used by the symbol ring.
//
// Drop-in for the reference's CSharedMemSimple (CSharedMemSimple.hpp:70-140):
// same class name, constructor (uid, size), master/slave ownership and error
// behaviour (perror + exit(EXIT_FAILURE) on any failure).  Both sides create
// or open the segment; only the side that called set_master_mode() unmaps and
// unlinks it on destruction.  Unlike the reference, no HAVE_UNISTD_H macro is
// needed (this build is Linux-only) and a failed mmap reports its errno.
#ifndef OFDM_CSHAREDMEMSIMPLE_HPP_
#define OFDM_CSHAREDMEMSIMPLE_HPP_

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <string>

class CSharedMemSimple {
  public:
    CSharedMemSimple(std::string shm_uid, unsigned int sizeInBytes)
        : name_(std::move(shm_uid)), bytes_(sizeInBytes) {
        fd_ = shm_open(name_.c_str(), O_CREAT | O_RDWR, S_IRUSR | S_IWUSR);
        if (fd_ == -1) die("shm_open");
        if (ftruncate(fd_, (off_t)bytes_) == -1) die("ftruncate");
        base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
        if (base_ == MAP_FAILED) die("mmap");
    }

    ~CSharedMemSimple() {
        if (!master_) return;  // only the owner tears the segment down
        munmap(base_, bytes_);
        shm_unlink(name_.c_str());
    }

    CSharedMemSimple(const CSharedMemSimple &) = delete;
    CSharedMemSimple &operator=(const CSharedMemSimple &) = delete;

    void set_master_mode() { master_ = true; }
    unsigned int nBytes() { return bytes_; }
    void *ptr() { return base_; }
    void info() {
        std::printf("SHM info: %s, %s\n", name_.c_str(), master_ ? "Master" : "Slave");
        std::printf("SHM bytes allocated: %u\n", nBytes());
    }

  private:
    [[noreturn]] static void die(const char *what) {
        std::perror(what);
        std::exit(EXIT_FAILURE);
    }

    std::string name_;
    unsigned int bytes_;
    int fd_ = -1;
    void *base_ = nullptr;
    bool master_ = false;
};

#endif  // OFDM_CSHAREDMEMSIMPLE_HPP_
