#include "shm_store.h"

#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <time.h>

#include <algorithm>
#include <stdexcept>

namespace ray_amd {

static const uint64_t kMagic = 0x52414D44534D5331ull;  // "RAMDSMS1"

struct Guard {
  ShmStore* s;
  explicit Guard(ShmStore* st) : s(st) { s->lock(); }
  ~Guard() { s->unlock(); }
};

static inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

static inline int bin_of(uint64_t n) {
  int b = 63 - __builtin_clzll(n | 1);
  return b < kNumBins ? b : kNumBins - 1;
}

static inline uint64_t hash_id(const uint8_t* id) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < kIdSize; ++i) {
    h ^= id[i];
    h *= 1099511628211ull;
  }
  return h;
}

ShmStore::ShmStore(const std::string& path, uint64_t size, bool create, uint64_t table_cap)
    : path_(path) {
  int fd;
  if (create) {
    fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
    if (fd < 0) throw std::runtime_error("shm open(create) failed: " + path);
    if (ftruncate(fd, (off_t)size) != 0) {
      close(fd);
      throw std::runtime_error("shm ftruncate failed");
    }
  } else {
    fd = open(path.c_str(), O_RDWR);
    if (fd < 0) throw std::runtime_error("shm open failed: " + path);
    struct stat st;
    fstat(fd, &st);
    size = (uint64_t)st.st_size;
  }
  void* p = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("shm mmap failed");
  base_ = (uint8_t*)p;
  size_ = size;
  hdr_ = (SegHeader*)base_;
  if (!create) {
    if (hdr_->magic != kMagic) throw std::runtime_error("shm segment not initialised");
    return;
  }
  // power-of-two table capacity
  uint64_t cap = 1024;
  while (cap < table_cap) cap <<= 1;
  memset(hdr_, 0, sizeof(SegHeader));
  hdr_->version = 1;
  hdr_->total_size = size;
  hdr_->table_cap = cap;
  hdr_->table_off = align_up(sizeof(SegHeader), 4096);
  hdr_->blocks_cap = cap * 2 + 64 * (1 + kMaxDevices);
  hdr_->blocks_off = align_up(hdr_->table_off + cap * sizeof(ObjEntry), 4096);
  hdr_->heap_off = align_up(hdr_->blocks_off + hdr_->blocks_cap * sizeof(Block), 4096);
  if (hdr_->heap_off + (1 << 20) > size) throw std::runtime_error("shm segment too small");
  memset(base_ + hdr_->table_off, 0, cap * sizeof(ObjEntry));
  Block* bl = blocks();
  memset(bl, 0, hdr_->blocks_cap * sizeof(Block));
  // free-record stack
  for (uint64_t i = 0; i < hdr_->blocks_cap; ++i) bl[i].next = (i + 1 < hdr_->blocks_cap) ? (uint32_t)(i + 2) : 0;
  hdr_->block_free_head = 1;
  pthread_mutexattr_t a;
  pthread_mutexattr_init(&a);
  pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
  pthread_mutex_init(&hdr_->mu, &a);
  pthread_mutexattr_destroy(&a);
  // host heap
  HeapHdr* h = &hdr_->heaps[0];
  h->base = hdr_->heap_off;
  h->size = (size - hdr_->heap_off) / kAlign * kAlign;
  uint32_t r = rec_alloc();
  Block& b = bl[r - 1];
  b.off = h->base;
  b.size = h->size;
  b.prev = b.next = 0;
  h->first = r;
  bin_push(h, r);
  h->valid = 1;
  __atomic_store_n(&hdr_->magic, kMagic, __ATOMIC_RELEASE);
}

bool ShmStore::populate(uint64_t off, uint64_t n, bool write) const {
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
  if (off >= size_) return true;
  n = std::min<uint64_t>(n, size_ - off);
  const uint64_t pg = 4096;
  const uint64_t b = off / pg * pg, e = align_up(off + n, pg);
  return madvise(base_ + b, e - b, write ? MADV_POPULATE_WRITE : MADV_POPULATE_READ) == 0;
}

ShmStore::~ShmStore() {
  if (base_) munmap(base_, size_);
}

void ShmStore::lock() {
  int rc = pthread_mutex_lock(&hdr_->mu);
  if (rc == EOWNERDEAD) pthread_mutex_consistent(&hdr_->mu);
}
void ShmStore::unlock() { pthread_mutex_unlock(&hdr_->mu); }

ObjEntry* ShmStore::table() const { return (ObjEntry*)(base_ + hdr_->table_off); }
Block* ShmStore::blocks() const { return (Block*)(base_ + hdr_->blocks_off); }
HeapHdr* ShmStore::heap(int device) {
  if (device < -1 || device >= kMaxDevices) throw std::runtime_error("bad device index");
  return &hdr_->heaps[device + 1];
}

uint32_t ShmStore::rec_alloc() {
  uint32_t r = hdr_->block_free_head;
  if (!r) throw std::runtime_error("object store block records exhausted");
  Block& b = blocks()[r - 1];
  hdr_->block_free_head = b.next;
  memset(&b, 0, sizeof(Block));
  b.in_use = 1;
  return r;
}
void ShmStore::rec_free(uint32_t r) {
  Block& b = blocks()[r - 1];
  memset(&b, 0, sizeof(Block));
  b.next = hdr_->block_free_head;
  hdr_->block_free_head = r;
}

void ShmStore::bin_push(HeapHdr* h, uint32_t r) {
  Block* bl = blocks();
  Block& b = bl[r - 1];
  int k = bin_of(b.size);
  b.free_ = 1;
  b.fprev = 0;
  b.fnext = h->bins[k];
  if (h->bins[k]) bl[h->bins[k] - 1].fprev = r;
  h->bins[k] = r;
}
void ShmStore::bin_remove(HeapHdr* h, uint32_t r) {
  Block* bl = blocks();
  Block& b = bl[r - 1];
  int k = bin_of(b.size);
  if (b.fprev) bl[b.fprev - 1].fnext = b.fnext;
  else h->bins[k] = b.fnext;
  if (b.fnext) bl[b.fnext - 1].fprev = b.fprev;
  b.free_ = 0;
  b.fprev = b.fnext = 0;
}

uint32_t ShmStore::heap_alloc(int device, uint64_t n) {
  HeapHdr* h = heap(device);
  if (!h->valid) return 0;
  n = align_up(n ? n : 1, kAlign);
  Block* bl = blocks();
  for (int k = bin_of(n); k < kNumBins; ++k) {
    for (uint32_t r = h->bins[k]; r; r = bl[r - 1].fnext) {
      if (bl[r - 1].size < n) continue;
      // take the split record BEFORE unlinking the free block: if the record pool is
      // exhausted the block is handed out whole instead of being orphaned
      uint32_t r2 = 0;
      if (bl[r - 1].size - n >= kAlign && hdr_->block_free_head) r2 = rec_alloc();
      bin_remove(h, r);
      if (r2) {  // split, remainder stays free
        Block& b1 = bl[r - 1];
        Block& b2 = bl[r2 - 1];
        b2.off = b1.off + n;
        b2.size = b1.size - n;
        b2.prev = r;
        b2.next = b1.next;
        if (b1.next) bl[b1.next - 1].prev = r2;
        b1.next = r2;
        b1.size = n;
        bin_push(h, r2);
      }
      h->used += bl[r - 1].size;
      return r;
    }
  }
  return 0;
}

void ShmStore::heap_free(int device, uint32_t r) {
  HeapHdr* h = heap(device);
  Block* bl = blocks();
  h->used -= bl[r - 1].size;
  // coalesce with next
  uint32_t nx = bl[r - 1].next;
  if (nx && bl[nx - 1].free_) {
    bin_remove(h, nx);
    bl[r - 1].size += bl[nx - 1].size;
    bl[r - 1].next = bl[nx - 1].next;
    if (bl[nx - 1].next) bl[bl[nx - 1].next - 1].prev = r;
    rec_free(nx);
  }
  uint32_t pv = bl[r - 1].prev;
  if (pv && bl[pv - 1].free_) {
    bin_remove(h, pv);
    bl[pv - 1].size += bl[r - 1].size;
    bl[pv - 1].next = bl[r - 1].next;
    if (bl[r - 1].next) bl[bl[r - 1].next - 1].prev = pv;
    rec_free(r);
    r = pv;
  }
  bin_push(h, r);
}

ObjEntry* ShmStore::find(const uint8_t* id) {
  ObjEntry* t = table();
  const uint64_t mask = hdr_->table_cap - 1;
  for (uint64_t i = hash_id(id) & mask, n = 0; n <= mask; i = (i + 1) & mask, ++n) {
    ObjEntry* e = &t[i];
    if (e->state == kEmpty) return nullptr;
    if (e->state != kTombstone && memcmp(e->id, id, kIdSize) == 0) return e;
  }
  return nullptr;
}

ObjEntry* ShmStore::insert_slot(const uint8_t* id) {
  ObjEntry* t = table();
  const uint64_t mask = hdr_->table_cap - 1;
  for (uint64_t i = hash_id(id) & mask, n = 0; n <= mask; i = (i + 1) & mask, ++n) {
    ObjEntry* e = &t[i];
    if (e->state == kEmpty || e->state == kTombstone) return e;
  }
  throw std::runtime_error("object table full");
}

// Linear probing with backward-shift deletion: after emptying slot i, every later entry
// of the probe run whose home slot is NOT cyclically in (i, j] moves back into the hole.
// The table never accumulates tombstones, so a miss stops at the first empty slot
// whatever the insert/delete history (a tombstone scheme decays to full-table scans).
void ShmStore::erase_slot(ObjEntry* e) {
  ObjEntry* t = table();
  const uint64_t mask = hdr_->table_cap - 1;
  uint64_t i = (uint64_t)(e - t);
  memset(&t[i], 0, sizeof(ObjEntry));  // kEmpty
  uint64_t j = i;
  for (;;) {
    j = (j + 1) & mask;
    if (t[j].state == kEmpty) break;
    const uint64_t k = hash_id(t[j].id) & mask;
    const bool stays = (i <= j) ? (i < k && k <= j) : (i < k || k <= j);
    if (stays) continue;
    memcpy(&t[i], &t[j], sizeof(ObjEntry));
    memset(&t[j], 0, sizeof(ObjEntry));
    i = j;
  }
}

static inline void check_id(const std::string& id) {
  if (id.size() != (size_t)kIdSize) throw std::invalid_argument("object id must be 20 bytes");
}

uint64_t ShmStore::create(const std::string& id, uint64_t data_size, uint64_t meta_size,
                          int device, bool pinned) {
  check_id(id);
  Guard g(this);
  const uint8_t* k = (const uint8_t*)id.data();
  if (find(k)) throw std::runtime_error("object already exists");
  // capacity check BEFORE the heap allocation (a full table must not leak the block)
  if (hdr_->num_objects * 10 >= hdr_->table_cap * 7) throw std::runtime_error("object table full");
  uint32_t r = heap_alloc(device, data_size + meta_size);
  if (!r) return UINT64_MAX;
  ObjEntry* e = insert_slot(k);
  memset(e, 0, sizeof(ObjEntry));
  memcpy(e->id, k, kIdSize);
  e->state = kCreated;
  e->device = device;
  e->block = r;
  e->offset = blocks()[r - 1].off;
  e->data_size = data_size;
  e->meta_size = meta_size;
  e->ref_count = 1;  // creator holds a pin until seal
  e->pinned = pinned ? 1 : 0;
  e->lru_tick = ++hdr_->lru_clock;
  e->creator_pid = (int32_t)getpid();
  hdr_->num_objects++;
  heap(device)->n_objects++;
  hdr_->stats_creates++;
  return e->offset;
}

bool ShmStore::seal(const std::string& id) {
  check_id(id);
  Guard g(this);
  ObjEntry* e = find((const uint8_t*)id.data());
  if (!e || e->state != kCreated) return false;
  __atomic_thread_fence(__ATOMIC_RELEASE);
  e->state = kSealed;
  e->ref_count -= 1;
  if (e->ref_count <= 0 && e->delete_pending) free_entry(e);
  return true;
}

// NOTE: moves other entries of the probe run (erase_slot): callers must not hold other
// ObjEntry pointers across a free_entry call — collect ids, then re-find.
void ShmStore::free_entry(ObjEntry* e) {
  heap_free(e->device, e->block);
  heap(e->device)->n_objects--;
  erase_slot(e);
  hdr_->num_objects--;
}

static void pin_add(ObjEntry* e, int pid, int d) {
  for (int i = 0; i < kPinPids; ++i)
    if (e->pin_pid[i] == pid && e->pin_cnt[i] > 0) {
      e->pin_cnt[i] += d;
      if (e->pin_cnt[i] <= 0) e->pin_pid[i] = e->pin_cnt[i] = 0;
      return;
    }
  if (d > 0)
    for (int i = 0; i < kPinPids; ++i)
      if (e->pin_cnt[i] == 0) {
        e->pin_pid[i] = pid;
        e->pin_cnt[i] = d;
        return;
      }
}

static void fill(const ObjEntry* e, ObjInfo* o) {
  o->id.assign((const char*)e->id, kIdSize);
  o->state = (int)e->state;
  o->device = e->device;
  o->offset = e->offset;
  o->data_size = e->data_size;
  o->meta_size = e->meta_size;
  o->ref_count = e->ref_count;
  o->lru_tick = e->lru_tick;
  o->pinned = e->pinned != 0;
  o->creator_pid = e->creator_pid;
}

bool ShmStore::get(const std::string& id, ObjInfo* out, bool pin) {
  check_id(id);
  Guard g(this);
  ObjEntry* e = find((const uint8_t*)id.data());
  if (!e || e->state != kSealed || e->delete_pending) return false;
  if (pin) {
    e->ref_count++;
    pin_add(e, (int)getpid(), 1);
  }
  e->lru_tick = ++hdr_->lru_clock;
  if (out) fill(e, out);
  return true;
}

bool ShmStore::release(const std::string& id) {
  check_id(id);
  Guard g(this);
  ObjEntry* e = find((const uint8_t*)id.data());
  if (!e) return false;
  if (e->ref_count > 0) {
    e->ref_count--;
    pin_add(e, (int)getpid(), -1);
  }
  if (e->ref_count == 0 && e->delete_pending) free_entry(e);
  return true;
}

bool ShmStore::remove(const std::string& id) {
  check_id(id);
  Guard g(this);
  ObjEntry* e = find((const uint8_t*)id.data());
  if (!e) return false;
  if (e->ref_count > 0) {
    e->delete_pending = 1;
    return true;
  }
  free_entry(e);
  return true;
}

bool ShmStore::contains(const std::string& id) {
  check_id(id);
  Guard g(this);
  ObjEntry* e = find((const uint8_t*)id.data());
  return e && e->state == kSealed && !e->delete_pending;
}

int ShmStore::state(const std::string& id) {
  check_id(id);
  Guard g(this);
  ObjEntry* e = find((const uint8_t*)id.data());
  return e ? (int)e->state : 0;
}

bool ShmStore::set_pinned(const std::string& id, bool pinned) {
  check_id(id);
  Guard g(this);
  ObjEntry* e = find((const uint8_t*)id.data());
  if (!e) return false;
  e->pinned = pinned ? 1 : 0;
  return true;
}

std::vector<std::string> ShmStore::evict(uint64_t bytes, int device) {
  Guard g(this);
  struct Cand {
    std::string id;
    uint64_t tick, size;
  };
  std::vector<Cand> cands;
  ObjEntry* t = table();
  for (uint64_t i = 0; i < hdr_->table_cap; ++i) {
    ObjEntry* e = &t[i];
    if (e->state == kSealed && e->device == device && e->ref_count == 0 && !e->pinned)
      cands.push_back({std::string((const char*)e->id, kIdSize), e->lru_tick,
                       e->data_size + e->meta_size});
  }
  std::sort(cands.begin(), cands.end(),
            [](const Cand& a, const Cand& b) { return a.tick < b.tick; });
  std::vector<std::string> out;
  uint64_t freed = 0;
  for (const Cand& c : cands) {
    if (freed >= bytes) break;
    ObjEntry* e = find((const uint8_t*)c.id.data());  // entries move on every free
    if (!e) continue;
    freed += c.size;
    out.push_back(c.id);
    free_entry(e);
    hdr_->stats_evictions++;
  }
  return out;
}

std::vector<std::string> ShmStore::spill_candidates(uint64_t bytes, int device) {
  Guard g(this);
  std::vector<ObjEntry*> cands;
  ObjEntry* t = table();
  for (uint64_t i = 0; i < hdr_->table_cap; ++i) {
    ObjEntry* e = &t[i];
    if (e->state == kSealed && e->device == device && e->ref_count == 0 && e->pinned)
      cands.push_back(e);
  }
  std::sort(cands.begin(), cands.end(),
            [](const ObjEntry* a, const ObjEntry* b) { return a->lru_tick < b->lru_tick; });
  std::vector<std::string> out;
  uint64_t acc = 0;
  for (ObjEntry* e : cands) {
    if (acc >= bytes) break;
    acc += e->data_size + e->meta_size;
    out.emplace_back((const char*)e->id, kIdSize);
  }
  return out;
}

std::vector<ObjInfo> ShmStore::list() {
  Guard g(this);
  std::vector<ObjInfo> out;
  ObjEntry* t = table();
  for (uint64_t i = 0; i < hdr_->table_cap; ++i) {
    if (t[i].state == kCreated || t[i].state == kSealed) {
      ObjInfo o;
      fill(&t[i], &o);
      out.push_back(o);
    }
  }
  return out;
}

void ShmStore::init_device_heap(int device, uint64_t arena_size) {
  Guard g(this);
  HeapHdr* h = heap(device);
  if (h->valid) return;
  memset(h, 0, sizeof(HeapHdr));
  h->base = 0;
  h->size = arena_size / kAlign * kAlign;
  uint32_t r = rec_alloc();
  Block& b = blocks()[r - 1];
  b.off = 0;
  b.size = h->size;
  h->first = r;
  bin_push(h, r);
  h->valid = 1;
}

bool ShmStore::device_heap_ready(int device) {
  Guard g(this);
  return heap(device)->valid != 0;
}

uint64_t ShmStore::used(int device) {
  Guard g(this);
  return heap(device)->used;
}
uint64_t ShmStore::capacity(int device) {
  Guard g(this);
  return heap(device)->size;
}
uint64_t ShmStore::num_objects() {
  Guard g(this);
  return hdr_->num_objects;
}
uint64_t ShmStore::evictions() {
  Guard g(this);
  return hdr_->stats_evictions;
}

uint64_t ShmStore::release_all_pins_of(int pid) {
  Guard g(this);
  ObjEntry* t = table();
  std::vector<std::string> drop;
  uint64_t changed = 0;
  for (uint64_t i = 0; i < hdr_->table_cap; ++i) {
    ObjEntry* e = &t[i];
    if (e->state != kCreated && e->state != kSealed) continue;
    bool touched = false;
    for (int k = 0; k < kPinPids; ++k)
      if (e->pin_pid[k] == pid && e->pin_cnt[k] > 0) {
        e->ref_count -= e->pin_cnt[k];
        if (e->ref_count < 0) e->ref_count = 0;
        e->pin_pid[k] = e->pin_cnt[k] = 0;
        touched = true;
      }
    // objects it created but never sealed are aborted; freed pins may complete a remove
    if ((e->state == kCreated && e->creator_pid == pid) ||
        (e->ref_count == 0 && e->delete_pending))
      drop.emplace_back((const char*)e->id, kIdSize);
    changed += touched;
  }
  for (const std::string& id : drop) {
    ObjEntry* e = find((const uint8_t*)id.data());
    if (e) {
      free_entry(e);
      ++changed;
    }
  }
  return changed;
}

bool ShmStore::abort(const std::string& id) {
  check_id(id);
  Guard g(this);
  ObjEntry* e = find((const uint8_t*)id.data());
  if (!e || e->state != kCreated) return false;
  free_entry(e);
  return true;
}

static int64_t mono_ms() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (int64_t)t.tv_sec * 1000 + t.tv_nsec / 1000000;
}

int64_t ShmStore::spill_request(int64_t bytes) {
  return __atomic_add_fetch(&hdr_->spill_want, bytes, __ATOMIC_ACQ_REL);
}

int64_t ShmStore::spill_take() { return __atomic_exchange_n(&hdr_->spill_want, 0, __ATOMIC_ACQ_REL); }

int64_t ShmStore::spill_inflight_add(int64_t d) {
  return __atomic_add_fetch(&hdr_->spills_inflight, d, __ATOMIC_ACQ_REL);
}

int64_t ShmStore::spill_inflight() const {
  return __atomic_load_n(&hdr_->spills_inflight, __ATOMIC_ACQUIRE);
}

void ShmStore::set_spiller(int64_t pid) {
  __atomic_store_n(&hdr_->spiller_beat_ms, mono_ms(), __ATOMIC_RELEASE);
  __atomic_store_n(&hdr_->spiller_pid, pid, __ATOMIC_RELEASE);
}

void ShmStore::spiller_beat() { __atomic_store_n(&hdr_->spiller_beat_ms, mono_ms(), __ATOMIC_RELEASE); }

int64_t ShmStore::live_spiller(int64_t max_age_ms) const {
  const int64_t pid = __atomic_load_n(&hdr_->spiller_pid, __ATOMIC_ACQUIRE);
  if (pid <= 0) return 0;
  const int64_t beat = __atomic_load_n(&hdr_->spiller_beat_ms, __ATOMIC_ACQUIRE);
  return mono_ms() - beat <= max_age_ms ? pid : 0;
}

uint64_t ShmStore::spilled_total_add(uint64_t n) {
  return __atomic_add_fetch(&hdr_->spilled_total, n, __ATOMIC_ACQ_REL);
}

}  // namespace ray_amd
