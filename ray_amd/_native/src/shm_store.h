// Shared-memory object store ("plasma" equivalent) for ray_amd.
//
// Reference behaviour: src/ray/object_manager/plasma/{store.cc,object_lifecycle_manager.cc,
// dlmalloc.cc,eviction_policy.cc}: create -> seal -> get/release, ref-counted pins,
// LRU eviction of unpinned sealed objects.
//
// Design difference: the reference runs the store inside the raylet and every
// create/get is an IPC round trip over a Unix socket. Here the allocator, the
// object table and the LRU clock live INSIDE the shared segment, guarded by a
// robust process-shared mutex, so any process on the node creates, seals and
// reads objects with a lock + a hash probe and zero IPC. Offsets (not pointers)
// are stored, since every process maps the segment at a different address.
//
// Block metadata is kept out-of-line (a record pool in the segment), so the
// very same allocator also manages the per-GPU HBM arenas (ops/csrc/gpu_arena.hip)
// whose bytes the host never touches: a GPU object is an entry whose `device`
// is >= 0 and whose `offset` is inside that GPU's arena.
#pragma once
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace ray_amd {

constexpr int kIdSize = 20;
constexpr int kMaxDevices = 16;
constexpr int kNumBins = 64;
constexpr uint64_t kAlign = 64;

// kTombstone is never written any more (deletion shifts the probe chain back); it is
// kept so that probes stay well defined on a segment created by an older build.
enum ObjState : uint32_t { kEmpty = 0, kCreated = 1, kSealed = 2, kTombstone = 3 };

constexpr int kPinPids = 4;  // reader pins tracked per process (crash cleanup)

struct ObjEntry {
  uint8_t id[kIdSize];
  uint32_t state;
  int32_t device;  // -1 = host heap, else GPU index (HBM arena)
  uint32_t block;  // block record index
  uint32_t pinned;  // primary copy pinned by its owner (spillable, not evictable)
  uint64_t offset;  // data offset: from segment start (host) or arena start (device)
  uint64_t data_size;
  uint64_t meta_size;
  int64_t ref_count;  // all pins (creator + readers)
  uint64_t lru_tick;
  uint32_t delete_pending;
  int32_t creator_pid;
  // Reader pins by process: the first kPinPids pinning processes are tracked so the
  // raylet can drop the pins of a process that died holding zero-copy views
  // (release_all_pins_of). Pins beyond that are counted in ref_count only.
  int32_t pin_pid[kPinPids];
  int32_t pin_cnt[kPinPids];
};

struct Block {
  uint64_t off, size;
  uint32_t prev, next;    // address-order neighbours (index+1, 0 = none)
  uint32_t fprev, fnext;  // free-list links (index+1)
  uint32_t free_;
  uint32_t in_use;  // record slot in use
};

struct HeapHdr {
  uint64_t base, size, used;
  uint32_t bins[kNumBins];  // free-list heads (index+1)
  uint32_t first;           // first block (index+1)
  uint32_t valid;
  uint64_t n_objects;
};

struct SegHeader {
  uint64_t magic, version, total_size;
  uint64_t table_cap, table_off;
  uint64_t blocks_cap, blocks_off;
  uint64_t heap_off;
  uint32_t block_free_head;  // free record stack (index+1)
  uint32_t pad0;
  uint64_t num_objects, lru_clock;
  uint64_t stats_evictions, stats_creates;
  pthread_mutex_t mu;
  HeapHdr heaps[1 + kMaxDevices];  // [0] host, [1+d] device d
  // Spill coordination (lock-free, every process of the node): puts that found the heap
  // full post the bytes they need; the node's spill thread (pid + heartbeat) takes them,
  // and counts the fused spill files it is writing, which puts wait on.
  int64_t spill_want;      // bytes requested by blocked puts, not yet taken
  int64_t spills_inflight; // fused spill writes in progress
  int64_t spiller_pid;     // the spill thread's process (0: none)
  int64_t spiller_beat_ms; // its last heartbeat (CLOCK_MONOTONIC ms)
  uint64_t spilled_total;  // bytes spilled since creation
};

struct ObjInfo {
  std::string id;
  int state = 0;
  int device = -1;
  uint64_t offset = 0, data_size = 0, meta_size = 0;
  int64_t ref_count = 0;
  uint64_t lru_tick = 0;
  bool pinned = false;
  int creator_pid = 0;
};

class ShmStore {
 public:
  ShmStore(const std::string& path, uint64_t size, bool create, uint64_t table_cap);
  ~ShmStore();

  uint8_t* base() const { return base_; }
  uint64_t size() const { return size_; }
  uint64_t heap_offset() const { return hdr_->heap_off; }

  // Page-table population for [off, off+n) of this process's mapping. A first write to a
  // page of the segment costs a fault per 4 KiB page in every process (tens of ms for a
  // 36 MiB image block); MADV_POPULATE_READ maps the already-allocated pages in one
  // syscall with fault-around (~10x cheaper), after which the copy runs at memcpy speed.
  // write=true (MADV_POPULATE_WRITE) also allocates and zeroes pages not yet backed:
  // the raylet runs that over the low end of the heap in the background so writers
  // rarely meet an unbacked page. Never modifies data. Returns false if unsupported.
  bool populate(uint64_t off, uint64_t n, bool write) const;

  // Returns data offset, or UINT64_MAX when the heap is full. Throws on duplicate id.
  uint64_t create(const std::string& id, uint64_t data_size, uint64_t meta_size, int device,
                  bool pinned);
  bool seal(const std::string& id);
  bool get(const std::string& id, ObjInfo* out, bool pin);
  bool release(const std::string& id);
  bool remove(const std::string& id);
  bool contains(const std::string& id);
  int state(const std::string& id);
  bool set_pinned(const std::string& id, bool pinned);
  std::vector<std::string> evict(uint64_t bytes, int device);
  std::vector<std::string> spill_candidates(uint64_t bytes, int device);
  std::vector<ObjInfo> list();
  void init_device_heap(int device, uint64_t arena_size);
  bool device_heap_ready(int device);
  uint64_t used(int device);
  uint64_t capacity(int device);
  uint64_t num_objects();
  uint64_t evictions();
  // spill coordination (see SegHeader)
  int64_t spill_request(int64_t bytes);
  int64_t spill_take();
  int64_t spill_inflight_add(int64_t d);
  int64_t spill_inflight() const;
  void set_spiller(int64_t pid);
  void spiller_beat();
  // the spill thread's pid if it beat within max_age_ms, else 0
  int64_t live_spiller(int64_t max_age_ms) const;
  uint64_t spilled_total_add(uint64_t n);
  // Drops every pin `pid` holds and aborts the objects it created but never sealed;
  // returns how many entries changed. Called by the raylet when a worker dies.
  uint64_t release_all_pins_of(int pid);
  // Abort an unsealed object (creator error path). False if absent or already sealed.
  bool abort(const std::string& id);

 private:
  ObjEntry* table() const;
  Block* blocks() const;
  ObjEntry* find(const uint8_t* id);
  ObjEntry* insert_slot(const uint8_t* id);
  HeapHdr* heap(int device);
  uint32_t rec_alloc();
  void rec_free(uint32_t r);
  void bin_push(HeapHdr* h, uint32_t r);
  void bin_remove(HeapHdr* h, uint32_t r);
  uint32_t heap_alloc(int device, uint64_t n);
  void erase_slot(ObjEntry* e);  // backward-shift deletion (no tombstones)
  void heap_free(int device, uint32_t r);
  void free_entry(ObjEntry* e);
  void lock();
  void unlock();
  friend struct Guard;

  std::string path_;
  uint8_t* base_ = nullptr;
  uint64_t size_ = 0;
  SegHeader* hdr_ = nullptr;
};

}  // namespace ray_amd
