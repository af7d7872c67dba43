// Framed message transport for ray_amd processes (driver, workers, raylet).
//
// Reference behaviour: Ray's core workers talk gRPC (src/ray/rpc/*) with a
// dedicated io_service thread per process. Here: one epoll thread per process
// owns every socket (Unix-domain on a node, TCP across nodes), reads
// length-prefixed frames, and hands complete frames to Python through a
// condition-variable queue; Python never holds the GIL while waiting and
// `send` writes directly from the calling thread when the socket is idle
// (falling back to the epoll thread's EPOLLOUT flush under back-pressure).
//
// Direct mode (the default; RAY_AMD_IO_THREAD=1 restores the epoll thread): there is no
// epoll thread, the thread calling poll() runs epoll_wait and reads the frames itself.
// Every received message then costs one thread wake-up instead of two (epoll thread ->
// condition variable -> poller); on a VM, where waking an idle vCPU costs 50-150 us, that
// is most of a small task's round trip. Every user of the loop polls it continuously from
// one thread (the core worker's dispatcher, the raylet / node agent main loops), which is
// what direct mode requires: a send that hits a full socket is flushed on the next poll.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

struct epoll_event;  // <sys/epoll.h>

namespace ray_amd {

enum EventType : int { kMessage = 0, kAccepted = 1, kClosed = 2 };

struct Event {
  int type;
  int conn;
  int aux;  // listener id for kAccepted
  std::string data;
};

struct Conn {
  int fd = -1;
  int id = 0;
  bool listener = false;
  std::mutex wmu;
  std::string out;        // pending bytes not yet written
  size_t out_pos = 0;
  bool want_out = false;
  std::string in;         // read buffer
  size_t in_pos = 0;
  bool closed = false;
};

class IOLoop {
 public:
  IOLoop();
  ~IOLoop();
  int listen_unix(const std::string& path);
  int listen_tcp(const std::string& host, int port, int* bound_port);
  int connect_unix(const std::string& path, int timeout_ms);
  int connect_tcp(const std::string& host, int port, int timeout_ms);
  bool send(int conn, const char* data, size_t n);
  bool send2(int conn, const char* a, size_t na, const char* b, size_t nb);
  void close_conn(int conn);
  // Wait up to timeout_ms (<0 forever) for at least one event; return up to max events.
  std::vector<Event> poll(int timeout_ms, size_t max_events);
  void wakeup();  // make a blocked poll() return (empty)
  void stop();
  size_t pending();

 private:
  void run();
  void process(const ::epoll_event* evs, int n);
  int add_fd(int fd, bool listener);
  void handle_read(std::shared_ptr<Conn> c);
  void handle_write(std::shared_ptr<Conn> c);
  void do_close(std::shared_ptr<Conn> c, bool emit);
  std::shared_ptr<Conn> get(int id);
  void push(Event&& e);
  bool write_locked(Conn* c, const char* a, size_t na, const char* b, size_t nb);

  int epfd_ = -1;
  int evfd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread th_;
  std::mutex cmu_;
  std::unordered_map<int, std::shared_ptr<Conn>> conns_;
  std::unordered_map<int, int> fd2id_;
  int next_id_ = 1;
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<Event> q_;
  int wake_pending_ = 0;
  bool direct_ = true;  // poll() drives epoll itself (no epoll thread)
  std::mutex ep_mu_;    // one epoll driver at a time in direct mode
};

}  // namespace ray_amd
