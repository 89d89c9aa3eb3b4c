// pubsub.hpp -- the reference's Go API (pubsub.go, client.go), mirrored in C++
// over the C ABI of psengine.h.
//
// go-libp2p-pubsub exposes NewTopicManager / NewTopic / PublishMessage /
// Subscribe / client.Messages / client.Close / Topic.Close.  This header keeps
// those names, argument meanings and error behaviour so that code written
// against the reference -- and its tests (pubsub_test.go) -- reads the same
// here.  What differs, and why:
//   * hosts are dense peer indices of one Network (one engine, one GPU) instead
//     of libp2p hosts; Host::Close() is the abrupt loss of a host
//     (pubsub_test.go:178) -- its parent's next write fails (subtree.go:333);
//   * the flood runs on the GPU for everything published since the last
//     flush; a subscriber's Messages() channel flushes before it is read, so
//     publish-then-read code works unchanged;
//   * a channel is an unbounded queue (the reference blocks at 16, client.go:79).
// Semantics of joins, repairs and orphans: DESIGN.md §2 (rules Q1-Q5).
#pragma once
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "psengine.h"

namespace pubsub {

constexpr int DefaultTreeWidth = 2;     // pubsub.go:16
constexpr int DefaultTreeMaxWidth = 5;  // pubsub.go:17

using Bytes = std::vector<uint8_t>;
using PeerID = uint32_t;

// Go's `error`: nil when code == 0 (PS_OK); `if (err) ...` tests non-nil.
struct Error {
  int code = PS_OK;
  std::string msg;
  explicit operator bool() const { return code != PS_OK; }
};

struct TreeOpts {  // pubsub.go:49-52
  int TreeWidth = DefaultTreeWidth;
  int TreeMaxWidth = DefaultTreeMaxWidth;
};

// Message and its wire codec: pubsub.go:122-153 (ps_msg_encode / ps_msg_decode)
enum MessageType : int32_t { Data = 0, Join = 1, Part = 2, Update = 3, State = 4 };
struct Message {
  MessageType Type = Data;
  Bytes data;
  std::vector<std::string> Peers;  // `json:"parents,omitempty"`
  int64_t TreeWidth = 0, TreeMaxWidth = 0, NumPeers = 0;
};
// writeMessage: appends json.NewEncoder(s).Encode(m)'s bytes to `stream`
Error writeMessage(std::string& stream, const Message& m);
// readMessage: decodes the next value at stream[*pos], advances *pos
Error readMessage(const std::string& stream, size_t* pos, Message* m);

class Network;
class Topic;
class client;
class Host;
class TopicManager;
class Channel;

// client.Messages() (client.go:26-28)
class Channel {
 public:
  // next payload, false when none is waiting (the reference's select falls to
  // its timeout) or the channel is closed
  bool Recv(Bytes* out);
  size_t Len();  // waiting payloads (after a flush)
  bool Closed() const { return closed_; }

 private:
  friend class Network;
  friend class TopicManager;
  friend class Topic;
  friend class client;
  friend class Host;
  Network* net_ = nullptr;
  std::deque<Bytes> q_;
  bool closed_ = false;
};

class client {  // client.go:16-22
 public:
  Channel& Messages() { return out_; }  // client.go:26-28
  Error Close();                        // client.go:30-34: Part + redistributeChildren
  PeerID Peer() const { return peer_; }

 private:
  friend class Network;
  friend class TopicManager;
  friend class Topic;
  friend class Host;
  friend class Channel;
  Network* net_ = nullptr;
  uint32_t topic_ = 0;
  PeerID peer_ = 0;
  bool open_ = true;
  Channel out_;
};

class Topic {  // pubsub.go:33-47
 public:
  Error PublishMessage(const Bytes& mes);  // pubsub.go:111-120
  Error Close();                           // pubsub.go:99-103
  const std::string& Title() const { return title_; }

 private:
  friend class Network;
  friend class TopicManager;
  friend class client;
  friend class Host;
  friend class Channel;
  Network* net_ = nullptr;
  uint32_t topic_ = 0;
  PeerID root_ = 0;
  std::string title_;
  bool open_ = true;
};

class Host {
 public:
  PeerID ID() const { return id_; }
  Error Close();  // abrupt: no Part; parents find out on their next write

 private:
  friend class Network;
  friend class TopicManager;
  friend class Topic;
  friend class client;
  friend class Channel;
  Network* net_ = nullptr;
  PeerID id_ = 0;
};

class TopicManager {  // pubsub.go:19-31
 public:
  // NewTopic (pubsub.go:54-97): a topic rooted at this manager's host
  Topic* NewTopic(const std::string& title, TreeOpts opts = TreeOpts{});
  // Subscribe (client.go:65-94): join the tree `topic` rooted at `itor`
  Error Subscribe(PeerID itor, const std::string& topic, client** out);
  std::map<std::string, Topic*> Topics;  // pubsub.go:20

 private:
  friend class Network;
  friend class Topic;
  friend class client;
  friend class Host;
  friend class Channel;
  Network* net_ = nullptr;
  PeerID h_ = 0;
};

// One engine: every host of a deployment, on one GPU.
class Network {
 public:
  Network(uint32_t n_hosts, uint32_t max_topics = 64, int device = 0);
  ~Network();
  Network(const Network&) = delete;
  Network& operator=(const Network&) = delete;

  Error status() const { return status_; }  // construction error (no GPU, ...)
  Host& host(PeerID i) { return hosts_[i]; }
  uint32_t size() const { return static_cast<uint32_t>(hosts_.size()); }
  TopicManager* NewTopicManager(Host& h);  // pubsub.go:26-31
  // Runs the flood for everything published so far and fills the channels.
  Error Flush();
  ps_engine* engine() { return e_; }

 private:
  friend class TopicManager;
  friend class Topic;
  friend class client;
  friend class Host;
  friend class Channel;
  Error err(int rc) const;

  ps_engine* e_ = nullptr;
  Error status_;
  uint32_t max_topics_ = 0;
  std::vector<Host> hosts_;
  std::vector<std::unique_ptr<TopicManager>> tms_;
  std::vector<std::unique_ptr<Topic>> topics_;
  std::vector<std::unique_ptr<client>> clients_;
  std::map<uint32_t, Bytes> payload_;     // msg id -> Data (the GPU moves ids)
  std::vector<uint32_t> pending_per_topic_;
  uint32_t pending_ = 0;
  bool solo_next_ = false;  // a host died: its first message runs on its own
  uint32_t window_ = 65536;
};

}  // namespace pubsub
