// pybind11 bindings: ray_amd._native._core
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <unistd.h>

#include <random>
#include <thread>
#include <vector>
#include <algorithm>
#include <cstring>

#include "channel.h"
#include "codec.h"
#include "io_loop.h"
#include "scheduler.h"
#include "shm_store.h"
#include "memory_monitor.h"

namespace py = pybind11;
using namespace ray_amd;

static py::object info_to_py(const ObjInfo& o) {
  py::dict d;
  d["id"] = py::bytes(o.id);
  d["state"] = o.state;
  d["device"] = o.device;
  d["offset"] = o.offset;
  d["data_size"] = o.data_size;
  d["meta_size"] = o.meta_size;
  d["ref_count"] = o.ref_count;
  d["lru_tick"] = o.lru_tick;
  d["pinned"] = o.pinned;
  d["creator_pid"] = o.creator_pid;
  return d;
}

static std::string as_str(const py::bytes& b) { return std::string(b); }

static thread_local std::mt19937_64* tl_rng = nullptr;

// A pinned view of a sealed object: exposes the buffer protocol and drops the
// reader pin when the last Python view of it dies (numpy arrays deserialized
// zero-copy from the store keep it alive through their base chain).
struct PinnedBuf {
  ShmStore* s = nullptr;
  std::string id;
  uint8_t* p = nullptr;
  uint64_t n = 0;
  bool readonly = true;
  bool pinned = false;
  ~PinnedBuf() {
    if (pinned && s) s->release(id);
  }
};

// Large copies into the shared-memory store are split over threads: one core's memcpy
// tops out near 10-12 GB/s, well under the socket's memory bandwidth.
static void parallel_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
  const uint64_t kMin = 8ull << 20;  // below this a single memcpy wins
  unsigned hw = std::thread::hardware_concurrency();
  unsigned nt = (unsigned)std::min<uint64_t>(n / kMin, std::min(8u, hw ? hw : 1u));
  if (nt <= 1) {
    memcpy(dst, src, n);
    return;
  }
  const uint64_t chunk = ((n / nt) + 4095) & ~4095ull;
  std::vector<std::thread> ts;
  for (unsigned t = 1; t < nt; ++t) {
    const uint64_t b = chunk * t;
    if (b >= n) break;
    const uint64_t e = std::min(n, b + chunk);
    ts.emplace_back([=] { memcpy(dst + b, src + b, e - b); });
  }
  memcpy(dst, src, std::min(n, chunk));
  for (auto& t : ts) t.join();
}

constexpr ssize_t kGilSendBytes = 256 << 10;

PYBIND11_MODULE(_core, m) {
  m.doc() = "ray_amd native runtime core: shm object store, frame I/O loop, scheduler";

  // ---- record codecs (Ray Data TFRecord read/write)
  m.def("crc32c", [](py::buffer b, uint32_t init) {
    py::buffer_info bi = b.request();
    const auto* p = static_cast<const uint8_t*>(bi.ptr);
    const size_t n = (size_t)bi.size * bi.itemsize;
    py::gil_scoped_release r;
    return crc32c(p, n, init);
  }, py::arg("data"), py::arg("init") = 0u);
  m.def("tfrecord_index", [](py::buffer b, bool verify) {
    py::buffer_info bi = b.request();
    const auto* p = static_cast<const uint8_t*>(bi.ptr);
    const size_t n = (size_t)bi.size * bi.itemsize;
    std::vector<std::pair<uint64_t, uint64_t>> idx;
    {
      py::gil_scoped_release r;
      idx = tfrecord_index(p, n, verify);
    }
    return idx;
  }, py::arg("data"), py::arg("verify") = true);
  m.def("tfrecord_encode", [](const std::vector<py::bytes>& recs) {
    std::string out;
    for (const auto& r : recs) {
      char* p;
      Py_ssize_t n;
      PyBytes_AsStringAndSize(r.ptr(), &p, &n);
      tfrecord_append(&out, reinterpret_cast<const uint8_t*>(p), (size_t)n);
    }
    return py::bytes(out);
  });

  // dst[:] = src (both contiguous buffers of equal byte size), split over threads with
  // the GIL released: staging a rollout batch into pinned host memory for the H2D copy
  m.def("copy_into", [](py::buffer dst, py::buffer src) {
    py::buffer_info d = dst.request(true), s = src.request();
    const uint64_t nd = (uint64_t)d.size * d.itemsize, ns = (uint64_t)s.size * s.itemsize;
    if (nd != ns) throw std::invalid_argument("copy_into: size mismatch");
    py::gil_scoped_release r;
    parallel_copy((uint8_t*)d.ptr, (const uint8_t*)s.ptr, nd);
  });

  // Strided row copy: for r < rows, dst[dst_off + r*dst_stride : +row_bytes] =
  // src[r*src_stride : +row_bytes] (byte offsets into two buffers), rows split over
  // threads with the GIL released. Assembles [T, B_total, ...] rollout batches straight
  // from per-runner [T, B_i, ...] fragments into pinned staging memory.
  m.def("copy_rows", [](py::buffer dst, uint64_t dst_off, uint64_t dst_stride, py::buffer src,
                        uint64_t src_stride, uint64_t rows, uint64_t row_bytes) {
    py::buffer_info d = dst.request(true), s = src.request();
    const uint64_t nd = (uint64_t)d.size * d.itemsize, ns = (uint64_t)s.size * s.itemsize;
    if (rows && (dst_off + (rows - 1) * dst_stride + row_bytes > nd ||
                 (rows - 1) * src_stride + row_bytes > ns))
      throw std::out_of_range("copy_rows: out of range");
    uint8_t* dp = (uint8_t*)d.ptr + dst_off;
    const uint8_t* sp = (const uint8_t*)s.ptr;
    py::gil_scoped_release r;
    const uint64_t total = rows * row_bytes;
    unsigned hw = std::thread::hardware_concurrency();
    unsigned nt = (unsigned)std::min<uint64_t>(total / (4ull << 20), std::min(8u, hw ? hw : 1u));
    if (nt > rows) nt = (unsigned)rows;
    auto work = [&](uint64_t r0, uint64_t r1) {
      for (uint64_t i = r0; i < r1; ++i) memcpy(dp + i * dst_stride, sp + i * src_stride, row_bytes);
    };
    if (nt <= 1) {
      work(0, rows);
      return;
    }
    std::vector<std::thread> ts;
    const uint64_t per = (rows + nt - 1) / nt;
    for (unsigned t = 1; t < nt; ++t) {
      const uint64_t r0 = per * t, r1 = std::min(rows, r0 + per);
      if (r0 < r1) ts.emplace_back(work, r0, r1);
    }
    work(0, std::min(rows, per));
    for (auto& t : ts) t.join();
  });

  m.def("random_id", [](int n) {
    if (!tl_rng) {
      std::random_device rd;
      tl_rng = new std::mt19937_64(((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)getpid());
    }
    std::string s(n, '\0');
    for (int i = 0; i < n; i += 8) {
      uint64_t v = (*tl_rng)();
      for (int j = 0; j < 8 && i + j < n; ++j) s[i + j] = (char)((v >> (8 * j)) & 0xff);
    }
    return py::bytes(s);
  });

  py::class_<ShmStore>(m, "ShmStore")
      .def(py::init<const std::string&, uint64_t, bool, uint64_t>(), py::arg("path"),
           py::arg("size") = 0, py::arg("create") = false, py::arg("table_cap") = 1 << 16)
      .def("create",
           [](ShmStore& s, py::bytes id, uint64_t n, uint64_t meta, int device, bool pinned) {
             std::string k = as_str(id);
             py::gil_scoped_release r;
             return s.create(k, n, meta, device, pinned);
           },
           py::arg("id"), py::arg("data_size"), py::arg("meta_size") = 0, py::arg("device") = -1,
           py::arg("pinned") = false)
      .def("seal", [](ShmStore& s, py::bytes id) { return s.seal(as_str(id)); })
      .def("get",
           [](ShmStore& s, py::bytes id, bool pin) -> py::object {
             ObjInfo o;
             bool ok;
             std::string k = as_str(id);
             {
               py::gil_scoped_release r;
               ok = s.get(k, &o, pin);
             }
             if (!ok) return py::none();
             return py::make_tuple(o.offset, o.data_size, o.meta_size, o.device);
           },
           py::arg("id"), py::arg("pin") = true)
      .def("get_buffer",
           [](ShmStore& s, py::bytes id, bool readonly) -> py::object {
             ObjInfo o;
             bool ok;
             std::string k = as_str(id);
             {
               py::gil_scoped_release r;
               ok = s.get(k, &o, true);
               // large objects are about to be read (deserialised views, H2D sources):
               // map their pages in one madvise rather than a read fault per 16 pages
               if (ok && o.data_size + o.meta_size >= (1u << 20))
                 s.populate(o.offset, o.data_size + o.meta_size, false);
             }
             if (!ok) return py::none();
             auto* b = new PinnedBuf();
             b->s = &s;
             b->id = k;
             b->p = s.base() + o.offset;
             b->n = o.data_size + o.meta_size;
             b->readonly = readonly;
             b->pinned = true;
             return py::cast(b, py::return_value_policy::take_ownership);
           },
           py::arg("id"), py::arg("readonly") = true, py::keep_alive<0, 1>())
      .def("info",
           [](ShmStore& s, py::bytes id) -> py::object {
             ObjInfo o;
             if (!s.get(as_str(id), &o, false)) return py::none();
             return info_to_py(o);
           })
      .def("release", [](ShmStore& s, py::bytes id) { return s.release(as_str(id)); })
      .def("remove", [](ShmStore& s, py::bytes id) { return s.remove(as_str(id)); })
      .def("contains", [](ShmStore& s, py::bytes id) { return s.contains(as_str(id)); })
      .def("state", [](ShmStore& s, py::bytes id) { return s.state(as_str(id)); })
      .def("set_pinned", [](ShmStore& s, py::bytes id, bool p) { return s.set_pinned(as_str(id), p); })
      .def("evict",
           [](ShmStore& s, uint64_t bytes, int device) {
             std::vector<py::bytes> out;
             for (auto& x : s.evict(bytes, device)) out.emplace_back(x);
             return out;
           },
           py::arg("bytes"), py::arg("device") = -1)
      .def("spill_candidates",
           [](ShmStore& s, uint64_t bytes, int device) {
             std::vector<py::bytes> out;
             for (auto& x : s.spill_candidates(bytes, device)) out.emplace_back(x);
             return out;
           },
           py::arg("bytes"), py::arg("device") = -1)
      .def("list",
           [](ShmStore& s) {
             py::list l;
             for (auto& o : s.list()) l.append(info_to_py(o));
             return l;
           })
      .def("buffer",
           [](ShmStore& s, uint64_t off, uint64_t n) {
             if (off + n > s.size()) throw std::out_of_range("buffer out of range");
             return py::memoryview::from_memory((void*)(s.base() + off), (ssize_t)n, false);
           })
      .def("address", [](ShmStore& s) { return (uintptr_t)s.base(); })
      .def("populate",
           [](ShmStore& s, uint64_t off, uint64_t n, bool write) {
             py::gil_scoped_release r;
             return s.populate(off, n, write);
           },
           py::arg("off"), py::arg("n"), py::arg("write") = false)
      .def_property_readonly("heap_offset", &ShmStore::heap_offset)
      .def("write",
           [](ShmStore& s, uint64_t off, py::buffer b) {
             py::buffer_info bi = b.request();
             uint64_t n = (uint64_t)bi.size * bi.itemsize;
             if (off + n > s.size()) throw std::out_of_range("write out of range");
             py::gil_scoped_release r;
             parallel_copy(s.base() + off, (const uint8_t*)bi.ptr, n);
           })
      .def("init_device_heap", &ShmStore::init_device_heap)
      .def("device_heap_ready", &ShmStore::device_heap_ready)
      .def("used", &ShmStore::used, py::arg("device") = -1)
      .def("capacity", &ShmStore::capacity, py::arg("device") = -1)
      .def("num_objects", &ShmStore::num_objects)
      .def("evictions", &ShmStore::evictions)
      .def("spill_request", &ShmStore::spill_request)
      .def("spill_take", &ShmStore::spill_take)
      .def("spill_inflight_add", &ShmStore::spill_inflight_add)
      .def("spill_inflight", &ShmStore::spill_inflight)
      .def("set_spiller", &ShmStore::set_spiller)
      .def("spiller_beat", &ShmStore::spiller_beat)
      .def("live_spiller", &ShmStore::live_spiller, py::arg("max_age_ms") = 2000)
      .def("spilled_total_add", &ShmStore::spilled_total_add)
      .def("release_all_pins_of", &ShmStore::release_all_pins_of)
      .def("abort", [](ShmStore& s, py::bytes id) { return s.abort(as_str(id)); })
      .def_property_readonly("size", &ShmStore::size);

  py::class_<PinnedBuf>(m, "PinnedBuf", py::buffer_protocol())
      .def_buffer([](PinnedBuf& b) {
        return py::buffer_info(b.p, 1, py::format_descriptor<uint8_t>::format(), 1,
                               {(ssize_t)b.n}, {(ssize_t)1}, b.readonly);
      })
      .def_property_readonly("size", [](PinnedBuf& b) { return b.n; })
      .def("release", [](PinnedBuf& b) {
        if (b.pinned && b.s) b.s->release(b.id);
        b.pinned = false;
      });

  py::class_<IOLoop>(m, "IOLoop")
      .def(py::init<>())
      .def("listen_unix", &IOLoop::listen_unix)
      .def("listen_tcp",
           [](IOLoop& io, const std::string& host, int port) {
             int bound = 0;
             int id = io.listen_tcp(host, port, &bound);
             return py::make_tuple(id, bound);
           })
      .def("connect_unix", &IOLoop::connect_unix, py::arg("path"), py::arg("timeout_ms") = 10000,
           py::call_guard<py::gil_scoped_release>())
      .def("connect_tcp", &IOLoop::connect_tcp, py::arg("host"), py::arg("port"),
           py::arg("timeout_ms") = 10000, py::call_guard<py::gil_scoped_release>())
      // Small frames are written with the GIL held: the socket is non-blocking (a full
      // socket buffers the rest for the epoll thread), so the write is a few-microsecond
      // syscall, while dropping the GIL around it hands the interpreter to another thread
      // and the sender then waits up to the switch interval to get it back (measured 75-90
      // us per send on the task-reply path of an 8-CPU node). Large frames release it.
      .def("send",
           [](IOLoop& io, int conn, py::bytes data) {
             char* p;
             ssize_t n;
             PyBytes_AsStringAndSize(data.ptr(), &p, &n);
             if (n < kGilSendBytes) return io.send(conn, p, (size_t)n);
             py::gil_scoped_release r;
             return io.send(conn, p, (size_t)n);
           })
      .def("send2",
           [](IOLoop& io, int conn, py::bytes a, py::buffer b) {
             char* p;
             ssize_t n;
             PyBytes_AsStringAndSize(a.ptr(), &p, &n);
             py::buffer_info bi = b.request();
             const size_t nb = (size_t)(bi.size * bi.itemsize);
             if ((size_t)n + nb < (size_t)kGilSendBytes)
               return io.send2(conn, p, (size_t)n, (const char*)bi.ptr, nb);
             py::gil_scoped_release r;
             return io.send2(conn, p, (size_t)n, (const char*)bi.ptr, nb);
           })
      .def("close", &IOLoop::close_conn)
      .def("poll",
           [](IOLoop& io, int timeout_ms, size_t max_events) {
             std::vector<Event> ev;
             {
               py::gil_scoped_release r;
               ev = io.poll(timeout_ms, max_events);
             }
             py::list out;
             for (auto& e : ev) {
               if (e.type == kMessage)
                 out.append(py::make_tuple(e.type, e.conn, py::bytes(e.data)));
               else
                 out.append(py::make_tuple(e.type, e.conn, e.aux));
             }
             return out;
           },
           py::arg("timeout_ms") = -1, py::arg("max_events") = 1024)
      .def("wakeup", &IOLoop::wakeup)
      .def("pending", &IOLoop::pending)
      .def("stop", &IOLoop::stop, py::call_guard<py::gil_scoped_release>());

  py::class_<Allocation>(m, "Allocation")
      .def(py::init<>())
      .def_readonly("node", &Allocation::node)
      .def_property_readonly("instances", [](const Allocation& a) {
        py::dict d;
        for (auto& kv : a.instances) {
          py::list l;
          for (auto& p : kv.second) l.append(py::make_tuple(p.first, (double)p.second / Scheduler::kUnit));
          d[py::str(kv.first)] = l;
        }
        return d;
      });

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<>())
      .def_readwrite("spread_threshold", &Scheduler::spread_threshold)
      .def("add_node", &Scheduler::add_node, py::arg("node_id"), py::arg("total"),
           py::arg("labels") = LabelMap())
      .def("remove_node", &Scheduler::remove_node)
      .def("set_draining", &Scheduler::set_draining)
      .def("nodes", &Scheduler::nodes)
      .def("total", &Scheduler::total)
      .def("available", &Scheduler::available)
      .def("cluster_total", &Scheduler::cluster_total)
      .def("cluster_available", &Scheduler::cluster_available)
      .def("labels", &Scheduler::labels)
      .def("pick_node", &Scheduler::pick_node, py::arg("req"), py::arg("strategy") = 0,
           py::arg("target") = "", py::arg("local") = "", py::arg("hard_labels") = LabelMap(),
           py::arg("soft_labels") = LabelMap())
      .def("feasible_anywhere", &Scheduler::feasible_anywhere, py::arg("req"),
           py::arg("hard_labels") = LabelMap())
      .def("allocate",
           [](Scheduler& s, const std::string& node, const ResMap& req) -> py::object {
             Allocation a;
             if (!s.allocate(node, req, &a)) return py::none();
             return py::cast(a);
           })
      .def("release", &Scheduler::release)
      .def("place_bundles",
           [](Scheduler& s, const std::vector<ResMap>& b, int strategy) {
             bool inf = false;
             auto nodes = s.place_bundles(b, strategy, &inf);
             return py::make_tuple(nodes, inf);
           })
      .def("commit_bundles", &Scheduler::commit_bundles)
      .def("remove_bundles", &Scheduler::remove_bundles)
      .def("pg_gpu_instances", &Scheduler::pg_gpu_instances);

  py::class_<MemoryMonitor>(m, "MemoryMonitor")
      .def(py::init<double, int64_t, std::string, std::string>(), py::arg("threshold") = 0.95,
           py::arg("min_free_bytes") = -1, py::arg("cgroup_root") = "/sys/fs/cgroup",
           py::arg("proc_root") = "/proc")
      .def("snapshot",
           [](const MemoryMonitor& mm) {
             MemorySnapshot s = mm.snapshot();
             return py::make_tuple(s.used, s.total, s.source);
           })
      .def("over_threshold",
           [](const MemoryMonitor& mm, uint64_t used, uint64_t total) {
             MemorySnapshot s;
             s.used = used;
             s.total = total;
             return mm.over_threshold(s);
           })
      .def("process_private_bytes", &MemoryMonitor::process_private_bytes,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("threshold", &MemoryMonitor::threshold);

  py::register_exception<ChannelClosed>(m, "ChannelClosedError");
  py::class_<ShmChannel>(m, "ShmChannel")
      .def(py::init<std::string, uint64_t, int, bool>(), py::arg("path"),
           py::arg("capacity") = 0, py::arg("num_readers") = 1, py::arg("create") = false)
      .def("write",
           [](ShmChannel& c, py::buffer b, double timeout) {
             py::buffer_info bi = b.request();
             const uint64_t n = (uint64_t)bi.size * (uint64_t)bi.itemsize;
             // fast path with the GIL held: releasing it costs a GIL hand-off to any
             // other Python thread of the process (tens of microseconds)
             if (n <= (64u << 10) && c.try_write((const char*)bi.ptr, n)) return true;
             py::gil_scoped_release r;
             return c.write((const char*)bi.ptr, n, timeout);
           },
           py::arg("data"), py::arg("timeout") = -1.0)
      .def("read",
           [](ShmChannel& c, int reader, double timeout) -> py::object {
             std::string out;
             bool ok = c.try_read(reader, &out);
             if (!ok && timeout != 0.0) {
               py::gil_scoped_release r;
               ok = c.read(reader, &out, timeout);
             }
             if (!ok) return py::none();
             return py::bytes(out);
           },
           py::arg("reader") = 0, py::arg("timeout") = -1.0)
      .def("close", &ShmChannel::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("closed", &ShmChannel::closed)
      .def_property_readonly("version", &ShmChannel::version)
      .def_property_readonly("capacity", &ShmChannel::capacity)
      .def_property_readonly("num_readers", &ShmChannel::num_readers)
      .def_static("set_spin_us", &ShmChannel::set_spin_us);
}
