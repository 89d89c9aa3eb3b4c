/*
 * psoracle.c -- CPU restatement of go-libp2p-pubsub v0 (TEST INFRASTRUCTURE).
 *
 * See psoracle.h for scope and pinning.  Every function cites the reference
 * lines it restates.  Quiescent rules used where the reference is timing
 * dependent (SURVEY.md F7, §7 "Hard parts"):
 *   Q1  State messages (subtree.go:137-147) are processed before the next
 *       join starts (the tests subscribe sequentially, pubsub_test.go:75-81).
 *   Q2  Go map iteration (subtree.go:163, 324, 358) is modelled as insertion
 *       order, except redirect ties: among the k>1 non-dead children of equal
 *       minimum size, the SplitMix64 stream picks index next() % k.
 *   Q3  Tree mutations caused by a message (lazy prune, failed-write repair)
 *       are applied after that message has reached every node (the message is
 *       not re-routed to repaired peers), in BFS order of the forwarding node.
 *   Q4  A write to a Part'ed (graceful) child succeeds; a write to a closed
 *       host fails on the first attempt (pubsub_test.go:178-186 / 301-311).
 *   Q5  Orphans (children of a departed node other than its last reported
 *       child, client.go:96-98 panics for them) receive nothing until they
 *       re-subscribe; their subtrees stay attached below them.
 */
#include "psoracle.h"
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

uint64_t or_splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t or_mix64(uint64_t x) {
  uint64_t s = x;
  return or_splitmix64(&s);
}

/* ---------------------------------------------------------------- tree --- */

/* one entry of subtree.children (subtree.go:36-44): the parent's view of a
 * child: its redirect counter `size`, the last State report `children`
 * (always a single peer, subtree.go:140) and the Part flag `dead`. */
typedef struct {
  uint32_t id;
  uint32_t reported;
  int64_t size;
  uint8_t dead;
} or_child;

typedef struct {
  or_child* v;
  uint32_t n, cap;
} or_clist;

struct or_tree {
  uint32_t n, root, W, MaxW;
  uint64_t rng;
  uint8_t* state;
  uint32_t* parent;
  or_clist* ch;
  /* scratch for BFS */
  uint32_t* q;
};

or_tree* or_tree_new(uint32_t n_peers, uint32_t root, uint32_t W, uint32_t MaxW,
                     uint64_t seed) {
  if (root >= n_peers) return NULL;
  or_tree* t = (or_tree*)calloc(1, sizeof(or_tree));
  if (!t) return NULL;
  t->n = n_peers;
  t->root = root;
  t->W = W;
  t->MaxW = MaxW;
  t->rng = seed;
  t->state = (uint8_t*)calloc(n_peers, 1);
  t->parent = (uint32_t*)malloc(sizeof(uint32_t) * n_peers);
  t->ch = (or_clist*)calloc(n_peers, sizeof(or_clist));
  t->q = (uint32_t*)malloc(sizeof(uint32_t) * n_peers);
  if (!t->state || !t->parent || !t->ch || !t->q) {
    or_tree_free(t);
    return NULL;
  }
  for (uint32_t i = 0; i < n_peers; i++) t->parent[i] = OR_NONE;
  t->state[root] = OR_IN;
  return t;
}

void or_tree_free(or_tree* t) {
  if (!t) return;
  if (t->ch)
    for (uint32_t i = 0; i < t->n; i++) free(t->ch[i].v);
  free(t->ch);
  free(t->state);
  free(t->parent);
  free(t->q);
  free(t);
}

static int clist_push(or_clist* L, uint32_t id) {
  if (L->n == L->cap) {
    uint32_t nc = L->cap ? L->cap * 2 : 4;
    or_child* nv = (or_child*)realloc(L->v, nc * sizeof(or_child));
    if (!nv) return OR_E_NOMEM;
    L->v = nv;
    L->cap = nc;
  }
  or_child* c = &L->v[L->n++];
  c->id = id;
  c->reported = OR_NONE;
  c->size = 0; /* &child{...} zero value, subtree.go:149 */
  c->dead = 0;
  return OR_OK;
}

static or_child* clist_find(or_clist* L, uint32_t id) {
  for (uint32_t i = 0; i < L->n; i++)
    if (L->v[i].id == id) return &L->v[i];
  return NULL;
}

/* handleJoin (subtree.go:110-154) + redirectJoin (subtree.go:156-194) + the
 * joiner's recursion in joinParents (subtree.go:241-307), starting at node x.
 * prio selects treeMaxWidth (subtree.go:111-114); redirected joins continue
 * with prio=false at the target (client.streamHandler -> joinNewPeer,
 * client.go:45-48, subtree.go:100-104). */
static int handle_join(or_tree* t, uint32_t x, uint32_t j, int prio) {
  for (;;) {
    uint32_t w = prio ? t->MaxW : t->W;
    or_clist* L = &t->ch[x];
    if (L->n >= w) {
      if (L->n == 0) return OR_E_NOPARENT; /* subtree.go:157-159 */
      int64_t mn = 10000000000ll;          /* subtree.go:161 */
      uint32_t k = 0;
      for (uint32_t i = 0; i < L->n; i++) {
        if (L->v[i].dead) continue;
        if (L->v[i].size < mn) {
          mn = L->v[i].size;
          k = 1;
        } else if (L->v[i].size == mn) {
          k++;
        }
      }
      if (k == 0) return OR_E_NOPARENT; /* minc == nil, subtree.go:172-174 */
      uint32_t pick = (k > 1) ? (uint32_t)(or_splitmix64(&t->rng) % k) : 0;
      or_child* minc = NULL;
      for (uint32_t i = 0; i < L->n; i++) {
        if (L->v[i].dead || L->v[i].size != mn) continue;
        if (pick == 0) {
          minc = &L->v[i];
          break;
        }
        pick--;
      }
      minc->size++; /* subtree.go:176-178 */
      uint32_t nx = minc->id;
      /* the joiner opens a stream to the redirect target (subtree.go:257);
       * a closed host refuses it and the join fails (subtree.go:302-304) */
      if (t->state[nx] == OR_FAILED) return OR_E_UNREACHABLE;
      x = nx;
      prio = 0;
      continue;
    }
    /* accept: welcome Update (subtree.go:121-132), child entry (149-152) */
    int rc = clist_push(L, j);
    if (rc) return rc;
    t->parent[j] = x;
    t->state[j] = OR_IN;
    /* State{Peers:[joiner], NumPeers: sub.size} to our parent
     * (subtree.go:137-147); sub.size is never written, so NumPeers = 0 and the
     * parent records size = 0 + 1 (subtree.go:57-61). */
    if (x != t->root && t->parent[x] != OR_NONE && t->state[x] == OR_IN) {
      or_child* me = clist_find(&t->ch[t->parent[x]], x);
      if (me) {
        me->size = 1;
        me->reported = j;
      }
    }
    return OR_OK;
  }
}

int or_tree_join(or_tree* t, uint32_t peer) {
  if (!t || peer >= t->n) return OR_E_INVAL;
  if (peer == t->root || t->state[peer] != OR_OUT) return OR_E_STATE;
  /* Subscribe dials the root (client.go:68-69) and joins there with
   * prio=false (Topic.AddPeer, pubsub.go:105-109). */
  return handle_join(t, t->root, peer, 0);
}

/* redistributeChildren (subtree.go:356-375) for the departed child entry `e`
 * of parent P, after the departed node `x` dropped its own children. Only the
 * last reported grandchild is re-attached, with prio=true. */
static int redistribute(or_tree* t, uint32_t P, uint32_t x, uint32_t reported) {
  /* x's children lose their upstream (client.go:103-112): all of them pause;
   * every one but the rescued one is orphaned for good (client.go:96-98). */
  or_clist* X = &t->ch[x];
  for (uint32_t i = 0; i < X->n; i++) {
    uint32_t c = X->v[i].id;
    if (c == reported) continue;
    if (t->state[c] == OR_IN) t->state[c] = OR_ORPHAN;
  }
  X->n = 0;
  if (reported == OR_NONE) return OR_OK;
  if (t->state[reported] != OR_IN || t->parent[reported] != x) {
    /* NewStream to a peer whose handler is gone fails (subtree.go:364-367) */
    return OR_OK;
  }
  t->state[reported] = OR_OUT; /* in flight: re-attached by handle_join */
  int rc = handle_join(t, P, reported, 1);
  if (rc != OR_OK) {
    t->state[reported] = OR_ORPHAN;
    t->parent[reported] = x;
  }
  return rc;
}

int or_tree_leave(or_tree* t, uint32_t x) {
  if (!t || x >= t->n) return OR_E_INVAL;
  if (x == t->root || t->state[x] != OR_IN) return OR_E_STATE;
  uint32_t P = t->parent[x];
  /* a Part written to a closed host is lost (subtree.go:89-92) */
  or_child* e = (P != OR_NONE && t->state[P] != OR_FAILED) ? clist_find(&t->ch[P], x) : NULL;
  /* subtree.Close: children's streams closed first (subtree.go:78-81), then
   * Part upstream (83-94); the parent marks dead and redistributes at once
   * (subtree.go:62-70).  The dead entry stays in the parent's map until the
   * parent's next forwardMessage prunes it (subtree.go:326-331). */
  t->state[x] = OR_DEAD;
  if (!e) {
    redistribute(t, P, x, OR_NONE);
    return OR_OK;
  }
  e->dead = 1;
  redistribute(t, P, x, e->reported);
  return OR_OK;
}

int or_tree_drop(or_tree* t, uint32_t x) {
  if (!t || x >= t->n) return OR_E_INVAL;
  if (x == t->root) return OR_E_STATE;
  if (t->state[x] != OR_IN && t->state[x] != OR_ORPHAN) return OR_E_STATE;
  /* host.Close(): nothing is sent; the parent notices on its next write. */
  t->state[x] = OR_FAILED;
  return OR_OK;
}

/* One message: forwardMessage at every reached node (subtree.go:319-354) and
 * delivery at each reached subscriber (client.go:124-130). */
int or_tree_message(or_tree* t, uint8_t* hop_out) {
  if (!t) return OR_E_INVAL;
  uint32_t n = t->n;
  if (hop_out) memset(hop_out, 0xFF, n);
  uint32_t* q = t->q;
  uint32_t qh = 0, qt = 0;
  q[qt++] = t->root;
  uint32_t level_end = qt;
  uint8_t h = 0;
  while (qh < qt) {
    if (qh == level_end) {
      level_end = qt;
    }
    uint32_t p = q[qh++];
    uint8_t hp = (p == t->root) ? 0 : (hop_out ? hop_out[p] : 0);
    or_clist* L = &t->ch[p];
    for (uint32_t i = 0; i < L->n; i++) {
      uint32_t c = L->v[i].id;
      if (t->state[c] != OR_IN) continue; /* dead / failed: no delivery */
      if (hop_out) hop_out[c] = (uint8_t)(hp + 1);
      q[qt++] = c;
    }
    (void)h;
  }
  /* lazy prune + failed-write repair at every forwarding node, BFS order */
  uint32_t nq = qt;
  for (uint32_t qi = 0; qi < nq; qi++) {
    uint32_t P = q[qi];
    or_clist* L = &t->ch[P];
    /* every failed child is repaired (subtree.go:342-349), however wide the
     * fan-out: the list holds up to L->n entries */
    uint32_t stack_f[64], stack_r[64];
    uint32_t* failed = stack_f;
    uint32_t* failed_rep = stack_r;
    if (L->n > 64) {
      failed = (uint32_t*)malloc((size_t)L->n * sizeof(uint32_t));
      failed_rep = (uint32_t*)malloc((size_t)L->n * sizeof(uint32_t));
      if (!failed || !failed_rep) {
        free(failed);
        free(failed_rep);
        return OR_E_NOMEM;
      }
    }
    uint32_t nf = 0;
    uint32_t w = 0;
    for (uint32_t i = 0; i < L->n; i++) {
      or_child e = L->v[i];
      if (e.dead) { /* delete(sub.children, c.id), subtree.go:329-331 */
        if (t->state[e.id] == OR_DEAD) {
          t->state[e.id] = OR_OUT;
          t->parent[e.id] = OR_NONE;
        }
        continue;
      }
      if (t->state[e.id] == OR_FAILED) { /* write error, subtree.go:333-336 */
        failed[nf] = e.id;
        failed_rep[nf] = e.reported;
        nf++;
        continue;
      }
      L->v[w++] = e;
    }
    L->n = w;
    for (uint32_t i = 0; i < nf; i++) /* subtree.go:342-349 */
      redistribute(t, P, failed[i], failed_rep[i]);
    if (failed != stack_f) {
      free(failed);
      free(failed_rep);
    }
  }
  return OR_OK;
}

void or_tree_parents(const or_tree* t, uint32_t* parent_out) {
  uint32_t n = t->n;
  for (uint32_t i = 0; i < n; i++) parent_out[i] = OR_NONE;
  uint32_t* q = t->q;
  uint32_t qh = 0, qt = 0;
  q[qt++] = t->root;
  while (qh < qt) {
    uint32_t p = q[qh++];
    or_clist* L = &t->ch[p];
    for (uint32_t i = 0; i < L->n; i++) {
      uint32_t c = L->v[i].id;
      if (t->state[c] != OR_IN) continue;
      parent_out[c] = p;
      q[qt++] = c;
    }
  }
}

uint32_t or_tree_state(const or_tree* t, uint32_t peer) {
  return peer < t->n ? t->state[peer] : OR_NONE;
}

uint32_t or_tree_n_children(const or_tree* t, uint32_t peer) {
  return peer < t->n ? t->ch[peer].n : 0;
}

/* ------------------------------------------------------------ hot path --- */

int64_t or_disseminate(uint32_t n, const uint32_t* row_ptr, const uint32_t* col,
                       uint32_t root, const uint8_t* live, uint32_t n_msgs,
                       const uint32_t* start_round, uint8_t* hop_out,
                       uint64_t* hist_out, uint32_t hist_len, int n_threads) {
  (void)start_round; /* hops are relative to the publish round */
  if (root >= n) return OR_E_INVAL;
  if (n_threads < 1) n_threads = 1;
  int64_t total = 0;
  int err = 0;
#pragma omp parallel num_threads(n_threads) reduction(+ : total)
  {
    uint32_t* stamp = (uint32_t*)calloc(n, sizeof(uint32_t));
    uint32_t* cur = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint32_t* nxt = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint64_t* hist = (uint64_t*)calloc(hist_len ? hist_len : 1, sizeof(uint64_t));
    if (!stamp || !cur || !nxt || !hist) {
#pragma omp atomic write
      err = 1;
    } else {
#pragma omp for schedule(dynamic, 1)
      for (int64_t mi = 0; mi < (int64_t)n_msgs; mi++) {
        uint32_t m = (uint32_t)mi;
        uint32_t tag = m + 1;
        /* PublishMessage: the root forwards, it is not a recipient
         * (pubsub.go:111-120; Topic has no out channel, pubsub.go:33-47) */
        stamp[root] = tag;
        uint32_t nc = 1, nn;
        cur[0] = root;
        uint32_t h = 0;
        uint8_t* hrow = hop_out ? hop_out + (size_t)m * n : NULL;
        while (nc) {
          h++;
          nn = 0;
          /* forwardMessage: every child of every node reached last round
           * (subtree.go:324-337); each child delivers then forwards
           * (client.go:124-130) -- one hop per tree edge. */
          for (uint32_t i = 0; i < nc; i++) {
            uint32_t p = cur[i];
            for (uint32_t e = row_ptr[p]; e < row_ptr[p + 1]; e++) {
              uint32_t c = col[e];
              if (!live[c] || stamp[c] == tag) continue;
              stamp[c] = tag;
              nxt[nn++] = c;
              if (hrow) hrow[c] = (uint8_t)(h > 254 ? 254 : h);
              if (h < hist_len) hist[h]++;
              total++;
            }
          }
          uint32_t* tmp = cur;
          cur = nxt;
          nxt = tmp;
          nc = nn;
        }
      }
      if (hist_out) {
#pragma omp critical
        for (uint32_t i = 0; i < hist_len; i++) hist_out[i] += hist[i];
      }
    }
    free(stamp);
    free(cur);
    free(nxt);
    free(hist);
  }
  if (err) return OR_E_NOMEM;
  return total;
}

/* The same hot path, restated the way the GPU engine computes it (CPU
 * baseline, bench.py): messages as bits, 64 per u64 word, and the rounds
 * level-synchronous -- round d writes every node of BFS level d, in parallel
 * over the level's nodes (OpenMP): a node whose parent was reached and which
 * is live receives new = row(parent) & ~seen(node) (seen is empty: each node
 * is reached once on a tree, subtree.go:324-337 / client.go:124-130).  Rows
 * are BFS-position major.
 *
 * Split in two like the GPU engine: or_levels_new does the per-topology work
 * (BFS numbering, row allocation, first touch of the rows) once, and
 * or_levels_run is one pass over a batch -- what the baseline times, as the
 * GPU's timed steps exclude the node-space build and reuse their buffers. */
struct or_levels {
  uint32_t n, qt, nl, W, n_msgs;
  uint32_t *order, *ppos, *lvl;
  uint64_t* rows;
  uint8_t* reached;
};

void or_levels_free(or_levels* L) {
  if (!L) return;
  free(L->order), free(L->ppos), free(L->lvl), free(L->rows), free(L->reached);
  free(L);
}

or_levels* or_levels_new(uint32_t n, const uint32_t* row_ptr, const uint32_t* col, uint32_t root,
                         uint32_t n_msgs) {
  if (root >= n || n_msgs == 0) return NULL;
  or_levels* L = (or_levels*)calloc(1, sizeof(or_levels));
  uint32_t* pos = (uint32_t*)malloc(sizeof(uint32_t) * n);
  if (!L || !pos) {
    free(L), free(pos);
    return NULL;
  }
  L->n = n;
  L->n_msgs = n_msgs;
  L->W = (n_msgs + 63) / 64;
  L->order = (uint32_t*)malloc(sizeof(uint32_t) * n);
  L->ppos = (uint32_t*)malloc(sizeof(uint32_t) * n);
  L->lvl = (uint32_t*)malloc(sizeof(uint32_t) * (n + 2));
  if (!L->order || !L->ppos || !L->lvl) {
    free(pos);
    or_levels_free(L);
    return NULL;
  }
  /* BFS numbering: order[], parent position, level starts */
  for (uint32_t i = 0; i < n; i++) pos[i] = OR_NONE;
  uint32_t qt = 0, nl = 0;
  L->order[qt] = root;
  L->ppos[qt] = OR_NONE;
  pos[root] = qt++;
  L->lvl[nl++] = 0;
  uint32_t lo = 0;
  while (lo < qt) {
    const uint32_t hi = qt;
    L->lvl[nl++] = hi;
    for (uint32_t i = lo; i < hi; i++)
      for (uint32_t e = row_ptr[L->order[i]]; e < row_ptr[L->order[i] + 1]; e++) {
        const uint32_t c = col[e];
        if (pos[c] != OR_NONE) continue;
        pos[c] = qt;
        L->order[qt] = c;
        L->ppos[qt++] = i;
      }
    lo = hi;
  }
  free(pos);
  L->qt = qt;
  L->nl = nl;
  L->rows = (uint64_t*)calloc((size_t)qt * L->W, sizeof(uint64_t)); /* zeroed: touched once here */
  L->reached = (uint8_t*)calloc(qt, 1);
  if (!L->rows || !L->reached) {
    or_levels_free(L);
    return NULL;
  }
  memset(L->rows, 0, sizeof(uint64_t) * (size_t)qt * L->W);
  return L;
}

/* One pass: every message of the batch from the root down every level.
 * Returns total deliveries (popcount of every new word). */
int64_t or_levels_run(or_levels* L, const uint8_t* live, int n_threads) {
  if (!L) return OR_E_INVAL;
  if (n_threads < 1) n_threads = 1;
  const uint32_t W = L->W;
  uint64_t* rows = L->rows;
  uint8_t* reached = L->reached;
  const uint32_t* ppos = L->ppos;
  const uint32_t* order = L->order;
  /* PublishMessage: the root holds the window's messages (not a recipient) */
  for (uint32_t w = 0; w < W; w++) rows[w] = ~0ull;
  if (L->n_msgs % 64) rows[W - 1] = (1ull << (L->n_msgs % 64)) - 1;
  reached[0] = 1;
  int64_t total = 0;
  for (uint32_t d = 1; d + 1 < L->nl; d++) {
    const int64_t a = L->lvl[d], b = L->lvl[d + 1];
#pragma omp parallel for num_threads(n_threads) schedule(static, 256) reduction(+ : total)
    for (int64_t u = a; u < b; u++) {
      const uint32_t p = ppos[u];
      reached[u] = 0;
      if (!reached[p] || !live[order[u]]) continue;
      reached[u] = 1;
      const uint64_t* src = rows + (size_t)p * W;
      uint64_t* dst = rows + (size_t)u * W;
      int64_t k = 0;
      for (uint32_t w = 0; w < W; w++) {
        const uint64_t nw = src[w]; /* & ~seen(u): empty for a fresh node */
        dst[w] = nw;
        k += __builtin_popcountll(nw);
      }
      total += k;
    }
  }
  return total;
}

int64_t or_levels_bits(uint32_t n, const uint32_t* row_ptr, const uint32_t* col, uint32_t root,
                       const uint8_t* live, uint32_t n_msgs, int n_threads) {
  if (root >= n) return OR_E_INVAL;
  if (n_msgs == 0) return 0;
  or_levels* L = or_levels_new(n, row_ptr, col, root, n_msgs);
  if (!L) return OR_E_NOMEM;
  const int64_t total = or_levels_run(L, live, n_threads);
  or_levels_free(L);
  return total;
}
