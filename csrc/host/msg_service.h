// Asynchronous point-to-point message service between the ranks of a job.
//
// Contract reproduced (not code): the closed boxps::PaddleShuffler used by the
// global data shuffle -- register_handler(consumer) -> service id,
// send_message_callback(client_id = service_id << 16 | rank, buf, len,
// ResultCallback*), wait_done(service_id), unregister_consumer, destroy
// (box_wrapper.h:672-673, data_set.cc:1906-1935, 2440-2604).  The reference
// library is not visible; this is a TCP full mesh:
//
//  * one outbound socket per peer, drained by a sender thread (FIFO per peer,
//    so an end-of-stream message always arrives after that peer's data);
//  * one inbound socket per peer, read by a receiver thread that runs the
//    target service's handler and then acknowledges the frame;
//  * a callback fires when the peer has ACKNOWLEDGED (handled) the message,
//    and wait_done(sid) blocks until every message sent by that service has
//    been handled on its destination;
//  * a peer whose socket fails (process died, connection reset) is marked
//    broken: its queued and in-flight frames are completed as FAILED (no
//    callback), further sends to it throw, and wait_done(sid) throws once the
//    service has no message left pending -- a lost peer fails the shuffle on
//    every rank instead of hanging it.
//
// Payloads are copied at send time, so the caller may reuse its buffer as soon
// as send_message returns (the reference clears its archive right after
// send_message_callback, data_set.cc:2487-2488).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace pbx {

class MsgService {
 public:
  using Handler = std::function<void(int src_rank, const char* buf, int64_t len)>;
  using Callback = std::function<void()>;

  MsgService(int rank, int world);
  ~MsgService();
  MsgService(const MsgService&) = delete;
  MsgService& operator=(const MsgService&) = delete;

  // bind + listen on host:port (port 0 = ephemeral); returns the bound port
  int listen(const std::string& host, int port);
  // connect the full mesh; endpoints[r] = "host:port" of rank r.  Blocks until
  // every peer's inbound connection has been accepted (timeout_s bound).
  void connect(const std::vector<std::string>& endpoints, double timeout_s = 60.0);

  // service ids are handed out in registration order, so ranks that register
  // their consumers in the same order agree on them (as in the reference)
  int register_handler(Handler h);
  void unregister_consumer(int sid);
  // client_id = (sid << 16) | dest_rank; len 0 is a legal (end-marker) message.
  // Throws if the destination peer is broken.
  void send_message(int client_id, const char* buf, int64_t len, Callback cb);
  // Blocks until nothing sent by sid is pending; throws if any of its
  // messages failed (broken peer).
  void wait_done(int sid);
  // ranks whose connection failed (empty when healthy)
  std::vector<int> broken_peers();
  // called (from a service thread, no service lock held) when a peer is lost
  using LossListener = std::function<void(int peer)>;
  int add_loss_listener(LossListener f);
  void remove_loss_listener(int id);
  void destroy();

  int rank() const { return rank_; }
  int world() const { return world_; }
  int64_t bytes_sent() const { return bytes_sent_.load(); }
  int64_t messages_handled() const { return handled_.load(); }

 private:
  struct Frame {
    uint32_t sid;
    uint64_t seq;
    std::string payload;
    Callback cb;
  };
  struct Peer {
    int out_fd = -1, in_fd = -1;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Frame> queue;
    std::map<uint64_t, std::pair<uint32_t, Callback>> inflight;  // seq -> (sid, cb)
    uint64_t next_seq = 0;
    bool broken = false;  // guarded by mu
    std::thread sender, acker, receiver;
  };
  void sender_loop(int peer);
  void acker_loop(int peer);
  void receiver_loop(int peer);
  Handler handler_for(uint32_t sid);
  void finish_one(uint32_t sid, Callback& cb);
  // mark a peer broken and fail everything queued / in flight to it
  void fail_peer(int peer, const char* why);

  int rank_, world_;
  int listen_fd_ = -1;
  std::vector<std::unique_ptr<Peer>> peers_;
  std::atomic<bool> stop_{false};
  bool connected_ = false;

  std::mutex hmu_;
  std::condition_variable hcv_;
  std::map<uint32_t, Handler> handlers_;
  uint32_t next_sid_ = 1;
  std::map<uint32_t, int64_t> pending_;  // sid -> messages not yet acknowledged
  std::map<uint32_t, std::string> failed_;  // sid -> first failure
  std::map<int, LossListener> listeners_;
  int next_listener_ = 1;

  std::atomic<int64_t> bytes_sent_{0}, handled_{0};
};

}  // namespace pbx
