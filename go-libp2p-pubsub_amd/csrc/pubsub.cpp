// pubsub.cpp -- the reference's Go API mirrored in C++ (include/pubsub.hpp)
// over the C ABI.  Host code only: every flood runs through ps_run.
#include "pubsub.hpp"

#include <cstring>

namespace pubsub {

// ------------------------------------------------------------------ codec ---
Error writeMessage(std::string& stream, const Message& m) {
  std::vector<const char*> peers;
  for (const auto& p : m.Peers) peers.push_back(p.c_str());
  ps_message cm{};
  cm.type = m.Type;
  cm.data = m.data.empty() ? nullptr : m.data.data();
  cm.data_len = m.data.size();
  cm.peers = peers.empty() ? nullptr : peers.data();
  cm.n_peers = peers.size();
  cm.tree_width = m.TreeWidth;
  cm.tree_max_width = m.TreeMaxWidth;
  cm.num_peers = m.NumPeers;
  size_t n = 0;
  int rc = ps_msg_encode(&cm, nullptr, 0, &n);
  if (rc != PS_OK && rc != PS_E_RANGE) return Error{rc, "encode"};
  const size_t at = stream.size();
  stream.resize(at + n);
  rc = ps_msg_encode(&cm, &stream[at], n, &n);
  if (rc != PS_OK) {
    stream.resize(at);
    return Error{rc, "encode"};
  }
  return Error{};
}

Error readMessage(const std::string& stream, size_t* pos, Message* m) {
  if (!pos || !m || *pos > stream.size()) return Error{PS_E_INVAL, "bad arguments"};
  const size_t left = stream.size() - *pos;
  // decoded fields are never longer than their encoding
  Bytes data(left + 1);
  std::string peers(left + 1, '\0');
  ps_message_buf b{};
  b.data = data.data();
  b.data_cap = data.size();
  b.peers = &peers[0];
  b.peers_cap = peers.size();
  size_t used = 0;
  const int rc = ps_msg_decode(stream.data() + *pos, left, &b, &used);
  if (rc != PS_OK) return Error{rc, left ? "malformed message" : "EOF"};
  *pos += used;
  m->Type = static_cast<MessageType>(b.type);
  m->data.assign(data.begin(), data.begin() + static_cast<long>(b.data_len));
  m->Peers.clear();
  for (size_t i = 0, o = 0; i < b.n_peers; ++i) {
    const size_t l = std::strlen(peers.c_str() + o);
    m->Peers.emplace_back(peers.c_str() + o, l);
    o += l + 1;
  }
  m->TreeWidth = b.tree_width;
  m->TreeMaxWidth = b.tree_max_width;
  m->NumPeers = b.num_peers;
  return Error{};
}

// ---------------------------------------------------------------- network ---
Network::Network(uint32_t n_hosts, uint32_t max_topics, int device) : max_topics_(max_topics) {
  ps_config cfg{};
  cfg.n_peers = n_hosts;
  cfg.n_topics = max_topics;
  cfg.tree_width = DefaultTreeWidth;
  cfg.tree_max_width = DefaultTreeMaxWidth;
  cfg.msg_window = window_;
  cfg.device = device;
  cfg.seed = 1;
  if (PS_ABI_CHECK() != PS_OK) {
    e_ = nullptr;
    status_ = Error{PS_E_INVAL, ps_last_error(nullptr)};
    return;
  }
  const int rc = ps_create(&cfg, &e_);
  if (rc != PS_OK) {
    e_ = nullptr;
    status_ = Error{rc, "ps_create failed (is a GPU visible?)"};
    return;
  }
  hosts_.resize(n_hosts);
  for (uint32_t i = 0; i < n_hosts; ++i) {
    hosts_[i].net_ = this;
    hosts_[i].id_ = i;
  }
  topics_.resize(max_topics);
  pending_per_topic_.assign(max_topics, 0);
}

Network::~Network() {
  if (e_) ps_destroy(e_);
}

Error Network::err(int rc) const {
  if (rc == PS_OK) return Error{};
  const char* m = e_ ? ps_last_error(e_) : "no engine";
  return Error{rc, m ? m : ""};
}

TopicManager* Network::NewTopicManager(Host& h) {
  tms_.emplace_back(new TopicManager());
  tms_.back()->net_ = this;
  tms_.back()->h_ = h.ID();
  return tms_.back().get();
}

Error Network::Flush() {
  if (!e_) return status_;
  if (pending_ == 0) return Error{};
  ps_stats st{};
  int rc = ps_run(e_, &st);
  pending_ = 0;
  std::fill(pending_per_topic_.begin(), pending_per_topic_.end(), 0u);
  if (rc != PS_OK) {
    payload_.clear();
    return err(rc);
  }
  // processMessages (client.go:124-128): every open subscriber's channel gets
  // what reached it, in arrival order
  std::vector<uint32_t> ids(64);
  for (auto& c : clients_) {
    if (!c->open_ || c->out_.closed_) continue;
    size_t n = 0;
    rc = ps_read_peer_messages(e_, c->topic_, c->peer_, ids.data(), ids.size(), &n);
    if (rc == PS_E_RANGE && n > ids.size()) {
      ids.resize(n);
      rc = ps_read_peer_messages(e_, c->topic_, c->peer_, ids.data(), ids.size(), &n);
    }
    if (rc != PS_OK) return err(rc);
    for (size_t k = 0; k < n; ++k) {
      auto it = payload_.find(ids[k]);
      if (it != payload_.end()) c->out_.q_.push_back(it->second);
    }
  }
  payload_.clear();
  return Error{};
}

// ------------------------------------------------------------------ hosts ---
Error Host::Close() {
  Network& N = *net_;
  if (!N.e_) return N.status_;
  Error e = N.Flush();  // what was published before the host died has flooded
  if (e) return e;
  for (auto& t : N.topics_) {
    if (!t || !t->open_) continue;
    const int rc = ps_topic_drop(N.e_, t->topic_, &id_, 1);
    if (rc == PS_OK) N.solo_next_ = true;  // PS_E_STATE: not subscribed there
  }
  for (auto& c : N.clients_)
    if (c->peer_ == id_) c->out_.closed_ = true;  // its read loop ends with the streams
  return Error{};
}

// ------------------------------------------------------------------ topic ---
Topic* TopicManager::NewTopic(const std::string& title, TreeOpts opts) {
  Network& N = *net_;
  if (!N.e_) return nullptr;
  uint32_t t = 0;
  while (t < N.max_topics_ && N.topics_[t] && N.topics_[t]->open_) ++t;
  if (t == N.max_topics_) return nullptr;
  if (ps_topic_create(N.e_, t, h_, static_cast<uint32_t>(opts.TreeWidth),
                      static_cast<uint32_t>(opts.TreeMaxWidth)) != PS_OK)
    return nullptr;
  N.topics_[t].reset(new Topic());
  Topic* T = N.topics_[t].get();
  T->net_ = net_;
  T->topic_ = t;
  T->root_ = h_;
  T->title_ = title;
  Topics[title] = T;  // pubsub.go:94
  return T;
}

Error Topic::PublishMessage(const Bytes& mes) {
  Network& N = *net_;
  if (!open_) return Error{PS_E_STATE, "topic closed"};
  uint32_t id = 0;
  const int rc = ps_publish(N.e_, &topic_, 1, &id);
  if (rc != PS_OK) return N.err(rc);
  N.payload_[id] = mes;
  ++N.pending_;
  // the first message after a host died runs on its own (it is lost below
  // the dead host, subtree.go:333-351), and a topic's window is bounded
  if (N.solo_next_ || ++N.pending_per_topic_[topic_] >= N.window_) {
    N.solo_next_ = false;
    return N.Flush();
  }
  return Error{};
}

Error Topic::Close() {
  Network& N = *net_;
  Error e = N.Flush();
  if (e) return e;
  const int rc = ps_topic_close(N.e_, topic_);
  if (rc != PS_OK) return N.err(rc);
  open_ = false;
  for (auto& tm : N.tms_)
    if (tm->h_ == root_) tm->Topics.erase(title_);  // pubsub.go:99-103
  return Error{};
}

// -------------------------------------------------------------- subscribe ---
Error TopicManager::Subscribe(PeerID itor, const std::string& topic, client** out) {
  Network& N = *net_;
  *out = nullptr;
  if (!N.e_) return N.status_;
  Topic* T = nullptr;
  for (auto& t : N.topics_)
    if (t && t->open_ && t->root_ == itor && t->title_ == topic) T = t.get();
  if (!T) return Error{PS_E_STATE, "protocol not supported"};  // NewStream fails (client.go:69-72)
  Error e = N.Flush();  // a later subscriber does not see earlier messages
  if (e) return e;
  int32_t st = 0;
  ps_topic_join(N.e_, T->topic_, &h_, 1, &st);
  if (st != PS_OK) return N.err(st);
  N.clients_.emplace_back(new client());
  client* c = N.clients_.back().get();
  c->net_ = net_;
  c->topic_ = T->topic_;
  c->peer_ = h_;
  c->out_.net_ = net_;
  *out = c;
  return Error{};
}

Error client::Close() {
  Network& N = *net_;
  if (!open_) return Error{};
  Error e = N.Flush();
  if (e) return e;
  const int rc = ps_topic_leave(N.e_, topic_, &peer_, 1);
  open_ = false;
  out_.closed_ = true;  // close(cli.out) when processMessages returns
  return N.err(rc);
}

// ---------------------------------------------------------------- channel ---
bool Channel::Recv(Bytes* out) {
  if (q_.empty() && !closed_ && net_) net_->Flush();
  if (q_.empty()) return false;
  *out = std::move(q_.front());
  q_.pop_front();
  return true;
}

size_t Channel::Len() {
  if (!closed_ && net_) net_->Flush();
  return q_.size();
}

}  // namespace pubsub
