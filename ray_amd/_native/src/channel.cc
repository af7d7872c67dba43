#include "channel.h"

#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <stdexcept>

namespace ray_amd {

int ShmChannel::spin_us_ = 50;

static inline double now_us() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static const uint64_t kChanMagic = 0x52414D4443484E31ull;  // "RAMDCHN1"

ShmChannel::ShmChannel(const std::string& path, uint64_t capacity, int num_readers, bool create)
    : path_(path), owner_(create) {
  if (create && (num_readers < 1 || num_readers > kChanMaxReaders))
    throw std::invalid_argument("channel needs 1..64 readers");
  int fd;
  if (create) {
    fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
    if (fd < 0) throw std::runtime_error("channel open(create) failed: " + path);
    map_size_ = sizeof(ChanHeader) + capacity;
    if (ftruncate(fd, (off_t)map_size_) != 0) {
      ::close(fd);
      throw std::runtime_error("channel ftruncate failed");
    }
  } else {
    fd = open(path.c_str(), O_RDWR);
    if (fd < 0) throw std::runtime_error("channel open failed: " + path);
    struct stat st;
    fstat(fd, &st);
    map_size_ = (uint64_t)st.st_size;
  }
  void* p = mmap(nullptr, map_size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("channel mmap failed");
  base_ = (uint8_t*)p;
  hdr_ = (ChanHeader*)base_;
  if (!create) {
    if (__atomic_load_n(&hdr_->magic, __ATOMIC_ACQUIRE) != kChanMagic)
      throw std::runtime_error("channel not initialised: " + path);
    return;
  }
  memset(hdr_, 0, sizeof(ChanHeader));
  pthread_mutexattr_t ma;
  pthread_mutexattr_init(&ma);
  pthread_mutexattr_setpshared(&ma, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&ma, PTHREAD_MUTEX_ROBUST);
  pthread_mutex_init(&hdr_->mu, &ma);
  pthread_mutexattr_destroy(&ma);
  pthread_condattr_t ca;
  pthread_condattr_init(&ca);
  pthread_condattr_setpshared(&ca, PTHREAD_PROCESS_SHARED);
  pthread_condattr_setclock(&ca, CLOCK_MONOTONIC);
  pthread_cond_init(&hdr_->readable, &ca);
  pthread_cond_init(&hdr_->writable, &ca);
  pthread_condattr_destroy(&ca);
  hdr_->capacity = capacity;
  hdr_->num_readers = (uint32_t)num_readers;
  __atomic_store_n(&hdr_->magic, kChanMagic, __ATOMIC_RELEASE);
}

ShmChannel::~ShmChannel() {
  if (base_) munmap(base_, map_size_);
}

void ShmChannel::lock() {
  int rc = pthread_mutex_lock(&hdr_->mu);
  if (rc == EOWNERDEAD) pthread_mutex_consistent(&hdr_->mu);
}
void ShmChannel::unlock() { pthread_mutex_unlock(&hdr_->mu); }

static bool deadline_of(double timeout_s, timespec* ts) {
  if (timeout_s < 0) return false;
  clock_gettime(CLOCK_MONOTONIC, ts);
  const double t = (double)ts->tv_sec + ts->tv_nsec * 1e-9 + timeout_s;
  ts->tv_sec = (time_t)t;
  ts->tv_nsec = (long)((t - (double)ts->tv_sec) * 1e9);
  return true;
}

bool ShmChannel::write(const char* data, uint64_t n, double timeout_s) {
  if (n > hdr_->capacity)
    throw std::length_error("channel payload of " + std::to_string(n) +
                            " bytes exceeds its capacity of " + std::to_string(hdr_->capacity));
  timespec ts;
  const bool timed = deadline_of(timeout_s, &ts);
  if (spin_us_ > 0) {
    const double t_end = now_us() + spin_us_;
    while (__atomic_load_n(&hdr_->reads_left, __ATOMIC_ACQUIRE) > 0 &&
           __atomic_load_n(&hdr_->version, __ATOMIC_ACQUIRE) > 0 &&
           !__atomic_load_n(&hdr_->closed, __ATOMIC_ACQUIRE) && now_us() < t_end)
      __builtin_ia32_pause();
  }
  lock();
  while (hdr_->version > 0 && hdr_->reads_left > 0 && !hdr_->closed) {
    hdr_->waiters_w++;
    int rc = timed ? pthread_cond_timedwait(&hdr_->writable, &hdr_->mu, &ts)
                   : pthread_cond_wait(&hdr_->writable, &hdr_->mu);
    if (rc == EOWNERDEAD) pthread_mutex_consistent(&hdr_->mu);
    hdr_->waiters_w--;
    if (rc == ETIMEDOUT) {
      unlock();
      return false;
    }
  }
  if (hdr_->closed) {
    unlock();
    throw ChannelClosed();
  }
  memcpy(base_ + sizeof(ChanHeader), data, n);
  hdr_->size = n;
  hdr_->reads_left = hdr_->num_readers;
  __atomic_store_n(&hdr_->version, hdr_->version + 1, __ATOMIC_RELEASE);
  const bool wake = hdr_->waiters_r > 0;
  unlock();
  if (wake) pthread_cond_broadcast(&hdr_->readable);
  return true;
}

bool ShmChannel::read(int reader, std::string* out, double timeout_s) {
  if (reader < 0 || reader >= (int)hdr_->num_readers) throw std::out_of_range("bad reader index");
  timespec ts;
  const bool timed = deadline_of(timeout_s, &ts);
  if (spin_us_ > 0) {
    const double t_end = now_us() + (timed ? std::min(spin_us_ * 1.0, timeout_s * 1e6) : spin_us_);
    while (__atomic_load_n(&hdr_->version, __ATOMIC_ACQUIRE) == hdr_->consumed[reader] &&
           !__atomic_load_n(&hdr_->closed, __ATOMIC_ACQUIRE) && now_us() < t_end)
      __builtin_ia32_pause();
  }
  lock();
  while (hdr_->consumed[reader] == hdr_->version && !hdr_->closed) {
    hdr_->waiters_r++;
    int rc = timed ? pthread_cond_timedwait(&hdr_->readable, &hdr_->mu, &ts)
                   : pthread_cond_wait(&hdr_->readable, &hdr_->mu);
    if (rc == EOWNERDEAD) pthread_mutex_consistent(&hdr_->mu);
    hdr_->waiters_r--;
    if (rc == ETIMEDOUT) {
      unlock();
      return false;
    }
  }
  if (hdr_->consumed[reader] == hdr_->version) {  // closed, nothing new
    unlock();
    throw ChannelClosed();
  }
  out->assign((const char*)base_ + sizeof(ChanHeader), hdr_->size);
  hdr_->consumed[reader] = hdr_->version;
  bool wake = false;
  if (hdr_->reads_left > 0) {
    __atomic_store_n(&hdr_->reads_left, hdr_->reads_left - 1, __ATOMIC_RELEASE);
    wake = hdr_->reads_left == 0 && hdr_->waiters_w > 0;
  }
  unlock();
  if (wake) pthread_cond_broadcast(&hdr_->writable);
  return true;
}

bool ShmChannel::try_write(const char* data, uint64_t n) {
  if (n > hdr_->capacity) return false;
  lock();
  if (hdr_->closed || (hdr_->version > 0 && hdr_->reads_left > 0)) {
    unlock();
    return false;
  }
  memcpy(base_ + sizeof(ChanHeader), data, n);
  hdr_->size = n;
  hdr_->reads_left = hdr_->num_readers;
  __atomic_store_n(&hdr_->version, hdr_->version + 1, __ATOMIC_RELEASE);
  const bool wake = hdr_->waiters_r > 0;
  unlock();
  if (wake) pthread_cond_broadcast(&hdr_->readable);
  return true;
}

bool ShmChannel::try_read(int reader, std::string* out) {
  if (reader < 0 || reader >= (int)hdr_->num_readers) return false;
  lock();
  if (hdr_->consumed[reader] == hdr_->version) {
    unlock();
    return false;
  }
  out->assign((const char*)base_ + sizeof(ChanHeader), hdr_->size);
  hdr_->consumed[reader] = hdr_->version;
  bool wake = false;
  if (hdr_->reads_left > 0) {
    __atomic_store_n(&hdr_->reads_left, hdr_->reads_left - 1, __ATOMIC_RELEASE);
    wake = hdr_->reads_left == 0 && hdr_->waiters_w > 0;
  }
  unlock();
  if (wake) pthread_cond_broadcast(&hdr_->writable);
  return true;
}

void ShmChannel::close() {
  lock();
  hdr_->closed = 1;
  pthread_cond_broadcast(&hdr_->readable);
  pthread_cond_broadcast(&hdr_->writable);
  unlock();
}

bool ShmChannel::closed() const { return __atomic_load_n(&hdr_->closed, __ATOMIC_ACQUIRE) != 0; }
uint64_t ShmChannel::version() const { return __atomic_load_n(&hdr_->version, __ATOMIC_ACQUIRE); }

}  // namespace ray_amd
