#include "io_loop.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <stdexcept>

namespace ray_amd {

static void set_nonblock(int fd) {
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
}

static void tune_socket(int fd, bool tcp) {
  int buf = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
  if (tcp) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
}

IOLoop::IOLoop() {
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (epfd_ < 0 || evfd_ < 0) throw std::runtime_error("epoll/eventfd failed");
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = 0;  // id 0 = wake fd
  epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
  const char* e = getenv("RAY_AMD_IO_THREAD");
  direct_ = !(e && e[0] == '1');
  if (!direct_) th_ = std::thread([this] { run(); });
}

IOLoop::~IOLoop() {
  stop();
  if (epfd_ >= 0) ::close(epfd_);
  if (evfd_ >= 0) ::close(evfd_);
}

void IOLoop::stop() {
  if (stop_.exchange(true)) return;
  uint64_t one = 1;
  ssize_t r = write(evfd_, &one, sizeof(one));
  (void)r;
  if (th_.joinable()) th_.join();
  std::lock_guard<std::mutex> g(cmu_);
  for (auto& kv : conns_) {
    if (kv.second->fd >= 0) ::close(kv.second->fd);
    kv.second->fd = -1;
    kv.second->closed = true;
  }
  conns_.clear();
  qcv_.notify_all();
}

int IOLoop::add_fd(int fd, bool listener) {
  set_nonblock(fd);
  auto c = std::make_shared<Conn>();
  c->fd = fd;
  c->listener = listener;
  {
    std::lock_guard<std::mutex> g(cmu_);
    c->id = next_id_++;
    conns_[c->id] = c;
    fd2id_[fd] = c->id;
  }
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP;
  ev.data.u64 = (uint64_t)c->id;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
  return c->id;
}

std::shared_ptr<Conn> IOLoop::get(int id) {
  std::lock_guard<std::mutex> g(cmu_);
  auto it = conns_.find(id);
  return it == conns_.end() ? nullptr : it->second;
}

int IOLoop::listen_unix(const std::string& path) {
  int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) throw std::runtime_error("socket failed");
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  if (path.size() >= sizeof(a.sun_path)) throw std::runtime_error("unix path too long: " + path);
  strncpy(a.sun_path, path.c_str(), sizeof(a.sun_path) - 1);
  unlink(path.c_str());
  if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0 || ::listen(fd, 1024) != 0) {
    ::close(fd);
    throw std::runtime_error("bind/listen failed: " + path + ": " + strerror(errno));
  }
  return add_fd(fd, true);
}

int IOLoop::listen_tcp(const std::string& host, int port, int* bound_port) {
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(port);
  inet_pton(AF_INET, host.c_str(), &a.sin_addr);
  if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0 || ::listen(fd, 1024) != 0) {
    ::close(fd);
    throw std::runtime_error("tcp bind/listen failed");
  }
  socklen_t len = sizeof(a);
  getsockname(fd, (sockaddr*)&a, &len);
  if (bound_port) *bound_port = ntohs(a.sin_port);
  return add_fd(fd, true);
}

int IOLoop::connect_unix(const std::string& path, int timeout_ms) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_un a{};
    a.sun_family = AF_UNIX;
    strncpy(a.sun_path, path.c_str(), sizeof(a.sun_path) - 1);
    if (::connect(fd, (sockaddr*)&a, sizeof(a)) == 0) {
      tune_socket(fd, false);
      return add_fd(fd, false);
    }
    ::close(fd);
    if (std::chrono::steady_clock::now() > deadline) return -1;
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
}

int IOLoop::connect_tcp(const std::string& host, int port, int timeout_ms) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(port);
    inet_pton(AF_INET, host.c_str(), &a.sin_addr);
    if (::connect(fd, (sockaddr*)&a, sizeof(a)) == 0) {
      tune_socket(fd, true);
      return add_fd(fd, false);
    }
    ::close(fd);
    if (std::chrono::steady_clock::now() > deadline) return -1;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
}

bool IOLoop::write_locked(Conn* c, const char* a, size_t na, const char* b, size_t nb) {
  // frame: u32 length (payload = a ++ b)
  uint32_t len = (uint32_t)(na + nb);
  char hdr[4];
  memcpy(hdr, &len, 4);
  if (c->closed || c->fd < 0) return false;
  if (!c->out.empty()) {  // keep ordering behind queued bytes
    c->out.append(hdr, 4);
    c->out.append(a, na);
    if (nb) c->out.append(b, nb);
    return true;
  }
  iovec iov[3] = {{hdr, 4}, {(void*)a, na}, {(void*)b, nb}};
  int niov = nb ? 3 : 2;
  size_t total = 4 + na + nb, done = 0;
  while (done < total) {
    ssize_t w = writev(c->fd, iov, niov);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      return false;
    }
    done += (size_t)w;
    size_t skip = (size_t)w;
    int k = 0;
    while (k < niov && skip >= iov[k].iov_len) { skip -= iov[k].iov_len; ++k; }
    if (k == niov) break;
    // shift iov
    int j = 0;
    for (int i = k; i < niov; ++i, ++j) iov[j] = iov[i];
    niov = j;
    iov[0].iov_base = (char*)iov[0].iov_base + skip;
    iov[0].iov_len -= skip;
  }
  if (done < total) {
    // queue remainder
    for (int i = 0; i < niov; ++i) c->out.append((const char*)iov[i].iov_base, iov[i].iov_len);
    c->out_pos = 0;
    if (!c->want_out) {
      c->want_out = true;
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP | EPOLLOUT;
      ev.data.u64 = (uint64_t)c->id;
      epoll_ctl(epfd_, EPOLL_CTL_MOD, c->fd, &ev);
    }
  }
  return true;
}

bool IOLoop::send(int conn, const char* data, size_t n) { return send2(conn, data, n, nullptr, 0); }

bool IOLoop::send2(int conn, const char* a, size_t na, const char* b, size_t nb) {
  auto c = get(conn);
  if (!c) return false;
  std::lock_guard<std::mutex> g(c->wmu);
  return write_locked(c.get(), a, na, b, nb);
}

void IOLoop::handle_write(std::shared_ptr<Conn> c) {
  std::lock_guard<std::mutex> g(c->wmu);
  while (c->out_pos < c->out.size()) {
    ssize_t w = ::write(c->fd, c->out.data() + c->out_pos, c->out.size() - c->out_pos);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) return;
      return;
    }
    c->out_pos += (size_t)w;
  }
  c->out.clear();
  c->out_pos = 0;
  c->want_out = false;
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP;
  ev.data.u64 = (uint64_t)c->id;
  epoll_ctl(epfd_, EPOLL_CTL_MOD, c->fd, &ev);
}

void IOLoop::push(Event&& e) {
  {
    std::lock_guard<std::mutex> g(qmu_);
    q_.push_back(std::move(e));
  }
  qcv_.notify_one();
}

void IOLoop::handle_read(std::shared_ptr<Conn> c) {
  char buf[1 << 16];
  bool eof = false;
  while (true) {
    ssize_t r = ::read(c->fd, buf, sizeof(buf));
    if (r > 0) {
      c->in.append(buf, (size_t)r);
      if ((size_t)r < sizeof(buf)) break;
      continue;
    }
    if (r == 0) { eof = true; break; }
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    eof = true;
    break;
  }
  // extract frames
  std::vector<Event> evs;
  while (c->in.size() - c->in_pos >= 4) {
    uint32_t len;
    memcpy(&len, c->in.data() + c->in_pos, 4);
    if (c->in.size() - c->in_pos - 4 < len) {
      // reserve for large frames
      if (c->in.capacity() < c->in_pos + 4 + len) c->in.reserve(c->in_pos + 4 + len);
      break;
    }
    Event e;
    e.type = kMessage;
    e.conn = c->id;
    e.aux = 0;
    e.data.assign(c->in.data() + c->in_pos + 4, len);
    c->in_pos += 4 + len;
    evs.push_back(std::move(e));
  }
  if (c->in_pos == c->in.size()) {
    c->in.clear();
    c->in_pos = 0;
  } else if (c->in_pos > (1 << 20)) {
    c->in.erase(0, c->in_pos);
    c->in_pos = 0;
  }
  if (!evs.empty()) {
    {
      std::lock_guard<std::mutex> g(qmu_);
      for (auto& e : evs) q_.push_back(std::move(e));
    }
    qcv_.notify_all();
  }
  if (eof) do_close(c, true);
}

void IOLoop::do_close(std::shared_ptr<Conn> c, bool emit) {
  {
    std::lock_guard<std::mutex> g(c->wmu);
    if (c->closed) return;
    c->closed = true;
    if (c->fd >= 0) {
      epoll_ctl(epfd_, EPOLL_CTL_DEL, c->fd, nullptr);
      ::close(c->fd);
    }
  }
  {
    std::lock_guard<std::mutex> g(cmu_);
    fd2id_.erase(c->fd);
    conns_.erase(c->id);
  }
  c->fd = -1;
  if (emit) push(Event{kClosed, c->id, 0, std::string()});
}

void IOLoop::close_conn(int conn) {
  auto c = get(conn);
  if (c) do_close(c, false);
}

void IOLoop::process(const epoll_event* evs, int n) {
  for (int i = 0; i < n; ++i) {
    int id = (int)evs[i].data.u64;
    if (id == 0) {
      uint64_t v;
      ssize_t r = ::read(evfd_, &v, sizeof(v));
      (void)r;
      continue;
    }
    auto c = get(id);
    if (!c) continue;
    if (c->listener) {
      while (true) {
        int fd = accept4(c->fd, nullptr, nullptr, SOCK_CLOEXEC);
        if (fd < 0) break;
        tune_socket(fd, false);
        int nid = add_fd(fd, false);
        push(Event{kAccepted, nid, c->id, std::string()});
      }
      continue;
    }
    if (evs[i].events & EPOLLOUT) handle_write(c);
    if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) handle_read(c);
  }
}

void IOLoop::run() {
  epoll_event evs[256];
  while (!stop_.load()) {
    int n = epoll_wait(epfd_, evs, 256, 200);
    if (n > 0) process(evs, n);
  }
}

std::vector<Event> IOLoop::poll(int timeout_ms, size_t max_events) {
  std::vector<Event> out;
  if (direct_) {
    {
      std::lock_guard<std::mutex> g(qmu_);
      if (wake_pending_ > 0) {
        wake_pending_--;
        while (!q_.empty() && out.size() < max_events) {
          out.push_back(std::move(q_.front()));
          q_.pop_front();
        }
        return out;
      }
      if (!q_.empty()) timeout_ms = 0;  // frames left from the last read: do not block
    }
    if (!stop_.load()) {
      std::lock_guard<std::mutex> ep(ep_mu_);
      epoll_event evs[256];
      int n = epoll_wait(epfd_, evs, 256, timeout_ms);
      if (n > 0) process(evs, n);
    }
    std::lock_guard<std::mutex> g(qmu_);
    if (wake_pending_ > 0) wake_pending_--;
    while (!q_.empty() && out.size() < max_events) {
      out.push_back(std::move(q_.front()));
      q_.pop_front();
    }
    return out;
  }
  std::unique_lock<std::mutex> lk(qmu_);
  auto ready = [this] { return !q_.empty() || wake_pending_ > 0 || stop_.load(); };
  if (timeout_ms < 0) qcv_.wait(lk, ready);
  else qcv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready);
  if (wake_pending_ > 0) wake_pending_--;
  while (!q_.empty() && out.size() < max_events) {
    out.push_back(std::move(q_.front()));
    q_.pop_front();
  }
  return out;
}

void IOLoop::wakeup() {
  {
    std::lock_guard<std::mutex> g(qmu_);
    wake_pending_++;
  }
  qcv_.notify_all();
  if (direct_) {  // a poller blocked in epoll_wait returns on the event fd
    uint64_t one = 1;
    ssize_t r = write(evfd_, &one, sizeof(one));
    (void)r;
  }
}

size_t IOLoop::pending() {
  std::lock_guard<std::mutex> g(qmu_);
  return q_.size();
}

}  // namespace ray_amd
