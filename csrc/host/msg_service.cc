#include "msg_service.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>

namespace pbx {

namespace {

constexpr uint32_t kMagic = 0x50425853;  // "PBXS"

struct FrameHeader {
  uint32_t magic;
  uint32_t sid;
  uint64_t seq;
  int64_t len;
};

bool write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += w;
    n -= (size_t)w;
  }
  return true;
}

bool read_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t r = ::recv(fd, c, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    c += r;
    n -= (size_t)r;
  }
  return true;
}

void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

bool split_endpoint(const std::string& ep, std::string* host, std::string* port) {
  const size_t c = ep.rfind(':');
  if (c == std::string::npos) return false;
  *host = ep.substr(0, c);
  *port = ep.substr(c + 1);
  return true;
}

}  // namespace

MsgService::MsgService(int rank, int world) : rank_(rank), world_(world) {
  if (world < 1 || rank < 0 || rank >= world || world > 0xffff) throw std::invalid_argument("MsgService: rank/world");
  for (int i = 0; i < world; ++i) peers_.emplace_back(new Peer());
}

MsgService::~MsgService() { destroy(); }

int MsgService::listen(const std::string& host, int port) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host.empty() ? nullptr : host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("MsgService::listen: cannot resolve " + host);
  listen_fd_ = ::socket(res->ai_family, res->ai_socktype, 0);
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (::bind(listen_fd_, res->ai_addr, res->ai_addrlen) != 0 || ::listen(listen_fd_, world_ + 8) != 0) {
    freeaddrinfo(res);
    throw std::runtime_error(std::string("MsgService::listen: ") + strerror(errno));
  }
  freeaddrinfo(res);
  sockaddr_in sa{};
  socklen_t sl = sizeof(sa);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&sa), &sl);
  return ntohs(sa.sin_port);
}

void MsgService::connect(const std::vector<std::string>& endpoints, double timeout_s) {
  if ((int)endpoints.size() != world_) throw std::invalid_argument("MsgService::connect: one endpoint per rank");
  if (world_ > 1 && listen_fd_ < 0) throw std::runtime_error("MsgService::connect: listen() first");
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds((int64_t)(timeout_s * 1000));
  // outbound: every peer already listens (endpoints are exchanged after
  // listen()), and the backlog holds our connection until the peer accepts
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    std::string host, port;
    if (!split_endpoint(endpoints[p], &host, &port)) throw std::invalid_argument("bad endpoint " + endpoints[p]);
    int fd = -1;
    while (fd < 0) {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) == 0 && res) {
        fd = ::socket(res->ai_family, res->ai_socktype, 0);
        if (::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
          ::close(fd);
          fd = -1;
        }
        freeaddrinfo(res);
      }
      if (fd < 0) {
        if (std::chrono::steady_clock::now() > deadline)
          throw std::runtime_error("MsgService::connect: timeout connecting to " + endpoints[p]);
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
    }
    tune(fd);
    const uint32_t hello[2] = {kMagic, (uint32_t)rank_};
    if (!write_all(fd, hello, sizeof(hello))) throw std::runtime_error("MsgService::connect: hello failed");
    peers_[p]->out_fd = fd;
  }
  // inbound: accept world-1 connections, identified by their hello
  for (int got = 0; got < world_ - 1;) {
    const int64_t left_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                                deadline - std::chrono::steady_clock::now()).count();
    if (left_ms <= 0) throw std::runtime_error("MsgService::connect: timeout waiting for peers");
    pollfd pf{listen_fd_, POLLIN, 0};
    if (::poll(&pf, 1, (int)std::min<int64_t>(left_ms, 1000)) <= 0) continue;
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) continue;
    tune(fd);
    uint32_t hello[2];
    if (!read_all(fd, hello, sizeof(hello)) || hello[0] != kMagic || (int)hello[1] >= world_ ||
        (int)hello[1] == rank_ || peers_[hello[1]]->in_fd >= 0) {
      ::close(fd);
      continue;
    }
    peers_[hello[1]]->in_fd = fd;
    ++got;
  }
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    Peer& pr = *peers_[p];
    pr.sender = std::thread(&MsgService::sender_loop, this, p);
    pr.acker = std::thread(&MsgService::acker_loop, this, p);
    pr.receiver = std::thread(&MsgService::receiver_loop, this, p);
  }
  connected_ = true;
}

int MsgService::register_handler(Handler h) {
  std::lock_guard<std::mutex> g(hmu_);
  const uint32_t sid = next_sid_++;
  if (sid > 0x7fff) throw std::runtime_error("MsgService: too many services");
  handlers_[sid] = std::move(h);
  pending_[sid] = 0;
  hcv_.notify_all();
  return (int)sid;
}

void MsgService::unregister_consumer(int sid) {
  // waits for our messages like wait_done, but never throws: a caller
  // unwinding from a failed shuffle must still be able to drop its handler
  {
    std::unique_lock<std::mutex> g(hmu_);
    hcv_.wait(g, [&] {
      auto it = pending_.find((uint32_t)sid);
      return stop_.load() || it == pending_.end() || it->second <= 0;
    });
  }
  std::lock_guard<std::mutex> g(hmu_);
  handlers_.erase((uint32_t)sid);
  pending_.erase((uint32_t)sid);
  failed_.erase((uint32_t)sid);
}

MsgService::Handler MsgService::handler_for(uint32_t sid) {
  // a peer may start sending before this rank registered the matching
  // consumer: hold the frame until it appears
  std::unique_lock<std::mutex> g(hmu_);
  // untimed wait (destroy() wakes it): a timed condition wait on the steady
  // clock is invisible to ThreadSanitizer's mutex tracking on this toolchain
  hcv_.wait(g, [&] { return stop_.load() || handlers_.count(sid) > 0; });
  auto it = handlers_.find(sid);
  return it == handlers_.end() ? Handler() : it->second;
}

void MsgService::finish_one(uint32_t sid, Callback& cb) {
  if (cb) cb();
  std::lock_guard<std::mutex> g(hmu_);
  auto it = pending_.find(sid);
  if (it != pending_.end()) --it->second;
  hcv_.notify_all();
}

void MsgService::fail_peer(int peer, const char* why) {
  Peer& p = *peers_[peer];
  std::vector<uint32_t> lost;  // sid of every frame that will never be acknowledged
  {
    std::lock_guard<std::mutex> g(p.mu);
    if (p.broken) return;
    p.broken = true;
    for (auto& f : p.queue) lost.push_back(f.sid);
    p.queue.clear();
    for (auto& e : p.inflight) lost.push_back(e.second.first);
    p.inflight.clear();
  }
  p.cv.notify_all();
  if (!stop_.load())
    fprintf(stderr, "[pbx msg] rank %d: peer %d lost (%s), %zu message(s) failed\n", rank_, peer, why, lost.size());
  std::vector<LossListener> ls;
  {
    std::lock_guard<std::mutex> g(hmu_);
    for (uint32_t sid : lost) {
      auto it = pending_.find(sid);
      if (it != pending_.end()) --it->second;
      if (!failed_.count(sid)) failed_[sid] = "message to rank " + std::to_string(peer) + " failed: " + why;
    }
    for (auto& e : listeners_) ls.push_back(e.second);
    hcv_.notify_all();
  }
  // listeners (e.g. a shuffle waiting for this peer's end-of-stream message)
  // run with none of this service's locks held
  for (auto& f : ls) f(peer);
}

int MsgService::add_loss_listener(LossListener f) {
  std::lock_guard<std::mutex> g(hmu_);
  const int id = next_listener_++;
  listeners_[id] = std::move(f);
  return id;
}

void MsgService::remove_loss_listener(int id) {
  std::lock_guard<std::mutex> g(hmu_);
  listeners_.erase(id);
}

std::vector<int> MsgService::broken_peers() {
  std::vector<int> out;
  for (int i = 0; i < world_; ++i) {
    if (i == rank_) continue;
    std::lock_guard<std::mutex> g(peers_[i]->mu);
    if (peers_[i]->broken) out.push_back(i);
  }
  return out;
}

void MsgService::send_message(int client_id, const char* buf, int64_t len, Callback cb) {
  const uint32_t sid = (uint32_t)client_id >> 16;
  const int dest = client_id & 0xffff;
  if (dest < 0 || dest >= world_) throw std::invalid_argument("MsgService::send_message: bad destination rank");
  {
    std::lock_guard<std::mutex> g(hmu_);
    if (!handlers_.count(sid)) throw std::invalid_argument("MsgService::send_message: unknown service id");
    ++pending_[sid];
  }
  if (dest == rank_) {  // loopback: handle inline
    Handler h = handler_for(sid);
    if (h) h(rank_, buf, len);
    ++handled_;
    finish_one(sid, cb);
    return;
  }
  if (!connected_) throw std::runtime_error("MsgService::send_message: not connected");
  Peer& p = *peers_[dest];
  Frame f{sid, 0, std::string(buf ? buf : "", buf ? (size_t)len : 0), std::move(cb)};
  bool broken;
  {
    std::lock_guard<std::mutex> g(p.mu);
    broken = p.broken;
    if (!broken) {
      f.seq = p.next_seq++;
      p.queue.push_back(std::move(f));
    }
  }
  if (broken) {
    {
      std::lock_guard<std::mutex> g(hmu_);
      --pending_[sid];
      hcv_.notify_all();
    }
    throw std::runtime_error("MsgService::send_message: rank " + std::to_string(dest) + " is lost");
  }
  p.cv.notify_one();
}

void MsgService::wait_done(int sid) {
  std::unique_lock<std::mutex> g(hmu_);
  hcv_.wait(g, [&] {
    auto it = pending_.find((uint32_t)sid);
    return stop_.load() || it == pending_.end() || it->second <= 0;
  });
  auto f = failed_.find((uint32_t)sid);
  if (f != failed_.end()) throw std::runtime_error("MsgService::wait_done(" + std::to_string(sid) + "): " + f->second);
}

void MsgService::sender_loop(int peer) {
  Peer& p = *peers_[peer];
  for (;;) {
    Frame f;
    {
      std::unique_lock<std::mutex> g(p.mu);
      p.cv.wait(g, [&] { return stop_.load() || !p.queue.empty(); });
      if (p.queue.empty()) return;
      f = std::move(p.queue.front());
      p.queue.pop_front();
      p.inflight[f.seq] = {f.sid, std::move(f.cb)};
    }
    FrameHeader h{kMagic, f.sid, f.seq, (int64_t)f.payload.size()};
    if (!write_all(p.out_fd, &h, sizeof(h)) || !write_all(p.out_fd, f.payload.data(), f.payload.size())) {
      fail_peer(peer, "send failed");
      return;
    }
    bytes_sent_ += (int64_t)(sizeof(h) + f.payload.size());
  }
}

void MsgService::acker_loop(int peer) {
  Peer& p = *peers_[peer];
  uint64_t seq;
  while (read_all(p.out_fd, &seq, sizeof(seq))) {
    std::pair<uint32_t, Callback> e;
    {
      std::lock_guard<std::mutex> g(p.mu);
      auto it = p.inflight.find(seq);
      if (it == p.inflight.end()) continue;
      e = std::move(it->second);
      p.inflight.erase(it);
    }
    finish_one(e.first, e.second);
  }
  // acknowledgements stopped: unless we are shutting down, the peer is gone
  if (!stop_.load()) fail_peer(peer, "connection closed");
}

void MsgService::receiver_loop(int peer) {
  Peer& p = *peers_[peer];
  std::string buf;
  FrameHeader h;
  while (read_all(p.in_fd, &h, sizeof(h))) {
    if (h.magic != kMagic || h.len < 0) {
      fprintf(stderr, "[pbx msg] rank %d: corrupt frame from %d\n", rank_, peer);
      return;
    }
    buf.resize((size_t)h.len);
    if (h.len && !read_all(p.in_fd, &buf[0], (size_t)h.len)) return;
    Handler fn = handler_for(h.sid);
    if (stop_.load()) return;
    if (fn) {
      fn(peer, h.len ? buf.data() : nullptr, h.len);
    } else if (!stop_.load()) {
      fprintf(stderr, "[pbx msg] rank %d: no consumer for service %u, dropped %lld bytes\n", rank_, h.sid,
              (long long)h.len);
    }
    ++handled_;
    if (!write_all(p.in_fd, &h.seq, sizeof(h.seq))) break;
  }
  if (!stop_.load()) fail_peer(peer, "inbound stream ended");
}

void MsgService::destroy() {
  if (stop_.exchange(true)) return;
  {
    std::lock_guard<std::mutex> g(hmu_);
    hcv_.notify_all();
  }
  for (auto& pp : peers_) {
    {
      std::lock_guard<std::mutex> g(pp->mu);
      pp->cv.notify_all();
    }
    if (pp->out_fd >= 0) ::shutdown(pp->out_fd, SHUT_RDWR);
    if (pp->in_fd >= 0) ::shutdown(pp->in_fd, SHUT_RDWR);
  }
  for (auto& pp : peers_) {
    if (pp->sender.joinable()) pp->sender.join();
    if (pp->acker.joinable()) pp->acker.join();
    if (pp->receiver.joinable()) pp->receiver.join();
    if (pp->out_fd >= 0) ::close(pp->out_fd);
    if (pp->in_fd >= 0) ::close(pp->in_fd);
    pp->out_fd = pp->in_fd = -1;
  }
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
}

}  // namespace pbx
