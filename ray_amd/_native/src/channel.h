// Mutable shared-memory channel: the transport of compiled DAGs.
//
// Reference behaviour: src/ray/core_worker/experimental_mutable_object_manager.cc and
// python/ray/experimental/channel/shared_memory_channel.py — a single-writer,
// N-reader mutable object that is overwritten in place once every reader has consumed
// the previous value (so a pipeline of actors exchanges values without any task
// submission, object-table entry or RPC per step).
//
// Design: one small /dev/shm file per channel holding a header (robust process-shared
// mutex, two process-shared condition variables on CLOCK_MONOTONIC, a version counter
// and per-reader consumed versions) followed by the payload bytes. Readers block in
// pthread_cond_timedwait (GIL released) after a short bounded spin on the version word
// (a woken futex waiter costs ~tens of microseconds of scheduler latency; a spinning
// reader sees the new version within a cache-line transfer).
#pragma once
#include <pthread.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

namespace ray_amd {

constexpr int kChanMaxReaders = 64;

struct ChannelClosed : std::runtime_error {
  ChannelClosed() : std::runtime_error("channel closed") {}
};

struct ChanHeader {
  uint64_t magic;
  pthread_mutex_t mu;
  pthread_cond_t readable;  // broadcast on write / close
  pthread_cond_t writable;  // broadcast when the last reader consumed a version
  uint64_t capacity;
  uint32_t num_readers;
  uint32_t closed;
  uint64_t version;  // 0 = nothing written yet
  uint64_t size;
  uint32_t reads_left;
  uint32_t waiters_r;  // readers blocked in pthread_cond_*wait (a writer skips the
  uint32_t waiters_w;  // futex wake when nobody sleeps)
  uint32_t pad;
  uint64_t consumed[kChanMaxReaders];
};

class ShmChannel {
 public:
  ShmChannel(const std::string& path, uint64_t capacity, int num_readers, bool create);
  ~ShmChannel();
  // Blocks until every reader consumed the previous value. Returns false on timeout.
  // Throws if closed or the payload exceeds the capacity.
  bool write(const char* data, uint64_t n, double timeout_s);
  // Non-blocking variants (no GIL release needed by the caller): false = would block.
  bool try_write(const char* data, uint64_t n);
  bool try_read(int reader, std::string* out);
  // Blocks until a version newer than this reader's last one exists. Returns false on
  // timeout; throws on a closed channel with nothing new to read.
  bool read(int reader, std::string* out, double timeout_s);
  void close();
  bool closed() const;
  uint64_t version() const;
  uint64_t capacity() const { return hdr_->capacity; }
  int num_readers() const { return (int)hdr_->num_readers; }
  static void set_spin_us(int us) { spin_us_ = us; }

 private:
  void lock();
  void unlock();
  std::string path_;
  uint8_t* base_ = nullptr;
  uint64_t map_size_ = 0;
  ChanHeader* hdr_ = nullptr;
  bool owner_ = false;
  static int spin_us_;
};

}  // namespace ray_amd
