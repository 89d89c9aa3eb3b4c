// pubsub_test.cpp -- the reference's own tests (pubsub_test.go) restated
// against the C++ mirror of its API (include/pubsub.hpp), running the flood on
// the GPU through libpsengine.so.  Same helpers (initPubsub, checkSystem,
// clearWaitingMessages), same skip sets, same assertions: every non-skipped
// subscriber receives exactly the published bytes, in order.
//
//   tests/cpp/bin/pubsub_test [test-name ...]      (exit 0 = all passed)
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <set>
#include <string>
#include <vector>

#include "pubsub.hpp"

using namespace pubsub;

namespace {

struct Fail {
  std::string msg;
};

#define REQUIRE(cond, ...)                          \
  do {                                              \
    if (!(cond)) {                                  \
      char b_[512];                                 \
      std::snprintf(b_, sizeof b_, __VA_ARGS__);    \
      throw Fail{b_};                               \
    }                                               \
  } while (0)

Bytes bytes(const std::string& s) { return Bytes(s.begin(), s.end()); }

// pubsub_test.go:63-82
Topic* initPubsub(Network& net, uint32_t count, std::vector<client*>& subs) {
  std::vector<TopicManager*> tms;
  for (uint32_t i = 0; i < count; ++i) tms.push_back(net.NewTopicManager(net.host(i)));
  const std::string title = "foobar";
  Topic* topic = tms[0]->NewTopic(title);
  REQUIRE(topic != nullptr, "NewTopic failed");
  for (uint32_t i = 1; i < count; ++i) {
    client* c = nullptr;
    Error err = tms[i]->Subscribe(net.host(0).ID(), title, &c);
    REQUIRE(!err, "Subscribe: %d %s", err.code, err.msg.c_str());
    subs.push_back(c);
  }
  return topic;
}

// pubsub_test.go:84-99
void clearWaitingMessages(std::vector<client*>& subs) {
  Bytes b;
  for (client* s : subs)
    while (s->Messages().Recv(&b)) {
    }
}

// pubsub_test.go:101-131
void checkSystem(Topic* t, std::vector<client*>& subs, const std::set<int>& skip, int mid) {
  char buf[64];
  std::snprintf(buf, sizeof buf, "message number %d", mid);
  const Bytes mes = bytes(buf);
  Error err = t->PublishMessage(mes);
  REQUIRE(!err, "PublishMessage: %s", err.msg.c_str());
  for (size_t i = 0; i < subs.size(); ++i) {
    if (skip.count(static_cast<int>(i))) continue;
    Bytes data;
    REQUIRE(subs[i]->Messages().Recv(&data), "Timeout waiting for peer %zu (message %d)", i, mid);
    REQUIRE(data == mes, "wrong data on node %zu. expected %s but got %s", i, buf,
            std::string(data.begin(), data.end()).c_str());
  }
}

void closeSubs(std::vector<client*>& subs) {
  for (client* c : subs) c->Close();
}

// pubsub_test.go:133-156
void TestBasicPubsub() {
  Network net(4);
  REQUIRE(!net.status(), "%s", net.status().msg.c_str());
  std::vector<client*> subs;
  Topic* topic = initPubsub(net, 4, subs);
  for (int i = 0; i < 10; ++i) checkSystem(topic, subs, {}, i);
  closeSubs(subs);
  REQUIRE(!topic->Close(), "Topic.Close");
}

// pubsub_test.go:158-202: hosts[1] (subs[0]) dies without a Part; the next
// message may be lost below it (subs 0 and 2 skipped), then the tree repairs
void TestNodesDropping() {
  Network net(4);
  std::vector<client*> subs;
  Topic* topic = initPubsub(net, 4, subs);
  checkSystem(topic, subs, {}, 0);
  REQUIRE(!net.host(1).Close(), "host close");
  checkSystem(topic, subs, {0, 2}, 1);
  clearWaitingMessages(subs);
  for (int i = 0; i < 10; ++i) checkSystem(topic, subs, {0}, i + 100);
  closeSubs(subs);
}

// pubsub_test.go:231-280: a lower node (hosts[3] = subs[2]) dies; either of
// its two children may miss the next message
void TestLowerNodesDropping() {
  Network net(8);
  std::vector<client*> subs;
  Topic* topic = initPubsub(net, 8, subs);
  checkSystem(topic, subs, {}, 0);
  REQUIRE(!net.host(3).Close(), "host close");
  checkSystem(topic, subs, {2, 5, 6}, 1);
  clearWaitingMessages(subs);
  for (int i = 0; i < 10; ++i) checkSystem(topic, subs, {2}, i + 100);
  closeSubs(subs);
}

// pubsub_test.go:282-325: subs[0] leaves with a Part
void TestNodesDroppingGracefully() {
  Network net(4);
  std::vector<client*> subs;
  Topic* topic = initPubsub(net, 4, subs);
  checkSystem(topic, subs, {}, 0);
  REQUIRE(!subs[0]->Close(), "client close");
  checkSystem(topic, subs, {0}, 1);
  clearWaitingMessages(subs);
  for (int i = 0; i < 10; ++i) checkSystem(topic, subs, {0}, i + 100);
  closeSubs(subs);
}

// BASELINE cfg1 through the API: 16 hosts, 1000 paced publishes, every
// subscriber gets every payload in order (pubsub_test.go:101-131 x 1000)
void TestPaced1000() {
  Network net(16);
  std::vector<client*> subs;
  Topic* topic = initPubsub(net, 16, subs);
  for (int i = 0; i < 1000; ++i) checkSystem(topic, subs, {}, i);
  closeSubs(subs);
}

// A burst: 300 publishes, then every channel drains in publish order
void TestBurstOrder() {
  Network net(40);
  std::vector<client*> subs;
  Topic* topic = initPubsub(net, 40, subs);
  for (int i = 0; i < 300; ++i) REQUIRE(!topic->PublishMessage(bytes("burst " + std::to_string(i))), "publish");
  for (size_t s = 0; s < subs.size(); ++s)
    for (int i = 0; i < 300; ++i) {
      Bytes b;
      REQUIRE(subs[s]->Messages().Recv(&b), "peer %zu missing message %d", s, i);
      REQUIRE(b == bytes("burst " + std::to_string(i)), "peer %zu out of order at %d", s, i);
    }
}

// Two topics rooted at different hosts; a host subscribed to both
void TestTwoTopics() {
  Network net(10);
  std::vector<TopicManager*> tms;
  for (uint32_t i = 0; i < 10; ++i) tms.push_back(net.NewTopicManager(net.host(i)));
  Topic* a = tms[0]->NewTopic("a");
  Topic* b = tms[5]->NewTopic("b", TreeOpts{3, 6});
  std::vector<client*> sa, sb;
  for (uint32_t i = 1; i < 10; ++i) {
    client* c = nullptr;
    REQUIRE(!tms[i]->Subscribe(0, "a", &c), "subscribe a");
    sa.push_back(c);
    if (i != 5) {
      REQUIRE(!tms[i]->Subscribe(5, "b", &c), "subscribe b");
      sb.push_back(c);
    }
  }
  client* none = nullptr;
  REQUIRE(tms[1]->Subscribe(0, "b", &none), "subscribe to a topic the host does not root must fail");
  REQUIRE(!a->PublishMessage(bytes("to a")) && !b->PublishMessage(bytes("to b")), "publish");
  Bytes x;
  for (client* c : sa) REQUIRE(c->Messages().Recv(&x) && x == bytes("to a") && !c->Messages().Recv(&x), "a");
  for (client* c : sb) REQUIRE(c->Messages().Recv(&x) && x == bytes("to b") && !c->Messages().Recv(&x), "b");
}

// writeMessage / readMessage (pubsub.go:122-134) over one stream
void TestWireCodec() {
  std::string stream;
  Message m1;
  m1.data = bytes("message number 0");
  Message m2;
  m2.Type = Update;
  m2.Peers = {"QmA", "Qm<B>"};
  m2.TreeWidth = 2;
  m2.TreeMaxWidth = 5;
  REQUIRE(!writeMessage(stream, m1) && !writeMessage(stream, m2), "encode");
  REQUIRE(stream == "{\"Type\":0,\"data\":\"bWVzc2FnZSBudW1iZXIgMA==\"}\n"
                    "{\"Type\":3,\"parents\":[\"QmA\",\"Qm\\u003cB\\u003e\"],\"treewidth\":2,\"treemaxwidth\":5}\n",
          "wire bytes: %s", stream.c_str());
  size_t pos = 0;
  Message r1, r2, r3;
  REQUIRE(!readMessage(stream, &pos, &r1) && !readMessage(stream, &pos, &r2), "decode");
  REQUIRE(r1.Type == Data && r1.data == m1.data && r1.Peers.empty(), "m1");
  REQUIRE(r2.Type == Update && r2.Peers == m2.Peers && r2.TreeWidth == 2 && r2.TreeMaxWidth == 5, "m2");
  REQUIRE(pos == stream.size() && readMessage(stream, &pos, &r3), "EOF after two values");
}

// INTEGRATION.md's cgo shim, call for call, through the C ABI: publish in
// batches, a run (ps_run) and a delivery to every subscriber
// (ps_read_peer_messages) whenever a topic's pending messages reach the
// window, and a final flush.  140,000 messages of one topic (more than two
// 65,536-message windows): every subscriber yields every message exactly
// once, in publish order (client.go:26-28,124-128).  Then the same burst as
// ONE run: ps_read_peer_messages holds only the last window -- the loss the
// shim's window flush avoids.
struct Shim {
  static constexpr uint32_t kWindow = 65536;
  ps_engine* e = nullptr;
  std::vector<size_t> pending;  // topic -> messages since the last run
  struct Sub {
    uint32_t topic, peer;
    std::vector<uint32_t> got;  // payload indices, in channel order
  };
  std::vector<Sub> subs;
  std::vector<uint32_t> payload;  // msg id - base -> payload index
  uint32_t base = 0;

  explicit Shim(uint32_t n_peers) {
    ps_config cfg{};
    cfg.n_peers = n_peers;
    cfg.n_topics = 1;
    cfg.tree_width = DefaultTreeWidth;
    cfg.tree_max_width = DefaultTreeMaxWidth;
    cfg.msg_window = kWindow;
    REQUIRE(ps_create(&cfg, &e) == PS_OK, "ps_create");
    pending.assign(1, 0);
  }
  ~Shim() { ps_destroy(e); }
  void flush() {
    if (pending[0] == 0) return;
    ps_stats st{};
    REQUIRE(ps_run(e, &st) == PS_OK, "ps_run: %s", ps_last_error(e));
    pending.assign(1, 0);
    std::vector<uint32_t> ids(1024);
    for (Sub& s : subs) {
      size_t n = 0;
      int rc = ps_read_peer_messages(e, s.topic, s.peer, ids.data(), ids.size(), &n);
      if (rc == PS_E_RANGE && n > ids.size()) {
        ids.resize(n);
        rc = ps_read_peer_messages(e, s.topic, s.peer, ids.data(), ids.size(), &n);
      }
      REQUIRE(rc == PS_OK, "ps_read_peer_messages: %s", ps_last_error(e));
      for (size_t k = 0; k < n; ++k) s.got.push_back(payload[ids[k] - base]);
    }
  }
  void publish(uint32_t topic, uint32_t first_payload, size_t count) {
    while (count) {
      const size_t k = std::min(count, kWindow - pending[topic]);
      std::vector<uint32_t> topics(k, topic);
      uint32_t first = 0;
      REQUIRE(ps_publish(e, topics.data(), k, &first) == PS_OK, "ps_publish");
      if (payload.empty()) base = first;
      for (size_t i = 0; i < k; ++i) {
        if (first + i - base >= payload.size()) payload.resize(first + i - base + 1);
        payload[first + i - base] = first_payload + static_cast<uint32_t>(i);
      }
      first_payload += static_cast<uint32_t>(k);
      pending[topic] += k;
      count -= k;
      if (pending[topic] == kWindow) flush();
    }
  }
};

void TestShimWindowFlush() {
  constexpr uint32_t kPeers = 48, kMsgs = 140000, kBatch = 1000;
  {
    Shim g(kPeers);
    REQUIRE(ps_topic_create(g.e, 0, 0, 0, 0) == PS_OK, "ps_topic_create");
    for (uint32_t p = 1; p < kPeers; ++p) {
      int32_t st = 0;
      REQUIRE(ps_topic_join(g.e, 0, &p, 1, &st) == PS_OK && st == PS_OK, "join %u", p);
      g.subs.push_back(Shim::Sub{0, p, {}});
    }
    for (uint32_t i = 0; i < kMsgs; i += kBatch) g.publish(0, i, kBatch);
    g.flush();
    for (const auto& s : g.subs) {
      REQUIRE(s.got.size() == kMsgs, "peer %u yielded %zu of %u messages", s.peer, s.got.size(), kMsgs);
      for (uint32_t i = 0; i < kMsgs; ++i) REQUIRE(s.got[i] == i, "peer %u: message %u out of order", s.peer, i);
    }
  }
  {  // one unflushed run of the same burst: only its last window is readable
    Shim g(kPeers);
    REQUIRE(ps_topic_create(g.e, 0, 0, 0, 0) == PS_OK, "ps_topic_create");
    for (uint32_t p = 1; p < kPeers; ++p) {
      int32_t st = 0;
      ps_topic_join(g.e, 0, &p, 1, &st);
    }
    std::vector<uint32_t> topics(kMsgs, 0);
    uint32_t first = 0;
    REQUIRE(ps_publish(g.e, topics.data(), kMsgs, &first) == PS_OK, "ps_publish");
    ps_stats st{};
    REQUIRE(ps_run(g.e, &st) == PS_OK && st.windows == 3, "ps_run");
    std::vector<uint32_t> ids(kMsgs);
    size_t n = 0;
    REQUIRE(ps_read_peer_messages(g.e, 0, 7, ids.data(), ids.size(), &n) == PS_OK, "read");
    REQUIRE(n == kMsgs - 2 * Shim::kWindow && ids[0] == first + 2 * Shim::kWindow, "last window only: %zu", n);
  }
}

}  // namespace

int main(int argc, char** argv) {
  const std::vector<std::pair<const char*, std::function<void()>>> tests = {
      {"TestWireCodec", TestWireCodec},
      {"TestBasicPubsub", TestBasicPubsub},
      {"TestNodesDropping", TestNodesDropping},
      {"TestLowerNodesDropping", TestLowerNodesDropping},
      {"TestNodesDroppingGracefully", TestNodesDroppingGracefully},
      {"TestPaced1000", TestPaced1000},
      {"TestBurstOrder", TestBurstOrder},
      {"TestTwoTopics", TestTwoTopics},
      {"TestShimWindowFlush", TestShimWindowFlush},
  };
  int failed = 0, ran = 0;
  for (const auto& t : tests) {
    bool want = argc == 1;
    for (int i = 1; i < argc; ++i) want |= std::strcmp(argv[i], t.first) == 0;
    if (!want) continue;
    ++ran;
    try {
      t.second();
      std::printf("--- PASS: %s\n", t.first);
    } catch (const Fail& f) {
      std::printf("--- FAIL: %s: %s\n", t.first, f.msg.c_str());
      ++failed;
    }
    std::fflush(stdout);
  }
  std::printf(failed ? "FAIL (%d of %d)\n" : "ok (%d of %d failed)\n", failed, ran);
  return failed ? 1 : 0;
}
