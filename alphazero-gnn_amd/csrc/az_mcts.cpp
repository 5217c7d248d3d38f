// az_mcts.cpp — native lock-step MCTS engine (see include/az_mcts.h for the contract).
//
// One tree per game slot: an open-addressing table from the 128-bit board key (two 64-bit
// occupancy masks, +1 and -1 stones) to nodes; per-node edge arrays (prior, visit count,
// typed Q) are allocated when a node first becomes a leaf (Vs, MCTS.py:163-165).  A search is
// a descent recorded as a path of (node, edge) and backed up once its value is known
// (terminal: immediately; new leaf: when the batched network result is fed back).
//
// Numeric parity with the reference (MCTS.py under NumPy 2 / NEP 50):
//   Qsa  <- (Nsa * Qsa + v) / (Nsa + 1)    (:228-233) with Python-int / Python-float /
//          np.float32 operands: int*f32 -> f32, float+f32 -> f32 (weak Python scalar cast to
//          f32 first), int+float -> float, int/int -> float, f32/int -> f32;
//   u    =  Q + cpuct * P[a] * sqrt(Ns) / (1 + Nsa)   or   cpuct * P[a] * sqrt(Ns + 1e-8)
//          in float64, left to right (:202-216), strict '>' keeps the first maximum;
//   P    =  float32 pi * int64 valids -> float64, divided by np.sum (pairwise summation).
#include "../../include/az_mcts.h"

#include <algorithm>
#include <new>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// ----------------------------------------------------------------------------- typed values
enum : uint8_t { T_INT = 0, T_F64 = 1, T_F32 = 2, T_NONE = 255 };

struct Val {
  double x;
  uint8_t tag;
};

inline Val vint(double x) { return {x == 0.0 ? 0.0 : x, T_INT}; }   // Python int has no -0
inline Val vneg(Val v) { return v.tag == T_INT ? vint(-v.x) : Val{-v.x, v.tag}; }

inline Val mul_n(long n, Val q) {                 // Nsa * Qsa, Nsa a Python int
  switch (q.tag) {
    case T_INT: return vint((double)n * q.x);
    case T_F64: return {(double)n * q.x, T_F64};
    default: return {(double)((float)n * (float)q.x), T_F32};
  }
}

inline Val add(Val a, Val b) {
  if (a.tag == T_F32 || b.tag == T_F32) return {(double)((float)a.x + (float)b.x), T_F32};
  if (a.tag == T_F64 || b.tag == T_F64) return {a.x + b.x, T_F64};
  return vint(a.x + b.x);
}

inline Val div_n(Val s, long d) {                 // ... / (Nsa + 1)
  if (s.tag == T_F32) return {(double)((float)s.x / (float)d), T_F32};
  return {s.x / (double)d, T_F64};                // int / int -> float (true division)
}

// NumPy's pairwise summation (numpy/_core/src/umath/loops_utils.h.src), float64.
double pairwise(const double* a, long n) {
  if (n < 8) {
    double r = 0.0;
    for (long i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    long i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  long n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise(a, n2) + pairwise(a + n2, n - n2);
}

// ----------------------------------------------------------------------------- rules
constexpr int kMaxA = 65;   // actions: n*n + 1 with n*n <= 64 cells

struct Key {
  uint64_t p, q;   // bit i = cell i (i = x*n + y) holds +1 / -1
  bool operator==(const Key& o) const { return p == o.p && q == o.q; }
};

inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t khash(const Key& k) { return mix64(k.p ^ mix64(k.q)); }

struct Rules {
  int game = 0, n = 0, A = 0, cells = 0;
  std::vector<uint64_t> lines;   // winning line masks
  uint64_t top = 0;              // Connect4: cells (x, n-1)
  uint64_t all = 0;

  bool init(int g, int nn) {
    if (nn < 1 || nn * nn > 64 || (g != AZM_GAME_CONNECT4 && g != AZM_GAME_TICTACTOE))
      return false;
    game = g;
    n = nn;
    cells = n * n;
    all = cells == 64 ? ~0ull : ((1ull << cells) - 1);
    auto bit = [&](int x, int y) { return 1ull << (x * n + y); };
    if (g == AZM_GAME_CONNECT4) {
      A = n + 1;
      int w = n < 4 ? n : 4;                     // min(4, n) in a row (Connect4Game.py:67-99)
      for (int x = 0; x < n; ++x) top |= bit(x, n - 1);
      const int dirs[4][2] = {{1, 0}, {0, 1}, {1, 1}, {1, -1}};
      for (auto& d : dirs)
        for (int x = 0; x < n; ++x)
          for (int y = 0; y < n; ++y) {
            int ex = x + d[0] * (w - 1), ey = y + d[1] * (w - 1);
            if (ex < 0 || ex >= n || ey < 0 || ey >= n) continue;
            uint64_t m = 0;
            for (int i = 0; i < w; ++i) m |= bit(x + d[0] * i, y + d[1] * i);
            lines.push_back(m);
          }
    } else {
      A = n * n + 1;                              // full rows, columns, two diagonals
      for (int j = 0; j < n; ++j) {
        uint64_t c = 0, r = 0;
        for (int i = 0; i < n; ++i) {
          c |= bit(i, j);
          r |= bit(j, i);
        }
        lines.push_back(c);
        lines.push_back(r);
      }
      uint64_t d1 = 0, d2 = 0;
      for (int i = 0; i < n; ++i) {
        d1 |= bit(i, i);
        d2 |= bit(i, n - 1 - i);
      }
      lines.push_back(d1);
      lines.push_back(d2);
    }
    index_lines();
    return true;
  }

  // The lines as (step, start mask) pairs: every line is w cells start + k step (k < w), so m
  // holds one iff some start bit of (m & m >> step & ... & m >> (w - 1) step) is set -- 4 x 3
  // shift-ands for Connect4 7x7 instead of a compare per line (88).  Lines of one step from
  // different directions (n = 2) merge exactly: the test is on the cells, not the direction.
  int wlen = 0, nsteps = -1;                     // -1: the plain per-line loop
  int steps[8] = {};
  uint64_t starts[8] = {};
  void index_lines() {
    nsteps = -1;
    if (lines.empty()) return;
    wlen = __builtin_popcountll(lines[0]);
    if (wlen < 2) return;
    int ns = 0;
    for (uint64_t l : lines) {
      const int s0 = __builtin_ctzll(l);
      const int st = __builtin_ctzll(l & (l - 1)) - s0;
      uint64_t want = 0;
      for (int k = 0; k < wlen; ++k) want |= 1ull << (s0 + k * st);
      if (want != l) return;                     // not an arithmetic run: keep the loop
      int j = 0;
      while (j < ns && steps[j] != st) ++j;
      if (j == ns) {
        if (ns == 8) return;
        steps[ns] = st;
        starts[ns++] = 0;
      }
      starts[j] |= 1ull << s0;
    }
    nsteps = ns;
  }

  bool run(uint64_t m) const {
    if (nsteps < 0) {
      for (uint64_t l : lines)
        if ((m & l) == l) return true;
      return false;
    }
    for (int j = 0; j < nsteps; ++j) {
      uint64_t a = m;
      for (int k = 1; k < wlen; ++k) a &= m >> (k * steps[j]);
      if (a & starts[j]) return true;
    }
    return false;
  }

  // getGameEnded(board, 1) (Connect4Game.py:169-183, TicTacToeGame.py:60-107)
  Val ended(const Key& k) const {
    if (run(k.p)) return vint(1);
    if (run(k.q)) return vint(-1);
    uint64_t occ = k.p | k.q;
    if (game == AZM_GAME_CONNECT4) {
      if ((occ & top) != top) return vint(0);
    } else if ((occ & all) != all) {
      return vint(0);
    }
    return {1e-4, T_F64};
  }

  // getValidMoves(board, 1) (Connect4Game.py:154-167, TicTacToeGame.py:44-58)
  void valids(const Key& k, uint8_t* v) const {
    uint64_t occ = k.p | k.q;
    bool any = false;
    if (game == AZM_GAME_CONNECT4) {
      for (int x = 0; x < n; ++x) {
        v[x] = !((occ >> (x * n + n - 1)) & 1);
        any |= v[x];
      }
    } else {
      for (int i = 0; i < cells; ++i) {
        v[i] = !((occ >> i) & 1);
        any |= v[i];
      }
    }
    v[A - 1] = !any;
  }

  // getCanonicalForm(getNextState(board, 1, a), -1): the mover's stone is +1, then the
  // board is negated for the opponent.  Pass (the last action) only negates.
  bool next(const Key& k, int a, Key* out) const {
    if (a == A - 1) {
      *out = {k.q, k.p};
      return true;
    }
    uint64_t occ = k.p | k.q, b;
    if (game == AZM_GAME_CONNECT4) {
      uint64_t col = ((occ >> (a * n)) & ((1ull << n) - 1));
      uint64_t free_ = ~col & ((1ull << n) - 1);
      if (!free_) return false;                  // "Column is full!" (Connect4Game.py:149)
      b = 1ull << (a * n + __builtin_ctzll(free_));
    } else {
      b = 1ull << a;
      if (occ & b) return false;
    }
    *out = {k.q, k.p | b};
    return true;
  }

  bool from_board(const int8_t* s, Key* k) const {
    k->p = k->q = 0;
    for (int i = 0; i < cells; ++i) {
      if (s[i] == 1) k->p |= 1ull << i;
      else if (s[i] == -1) k->q |= 1ull << i;
      else if (s[i] != 0) return false;
    }
    return true;
  }

  // 8 cells at a time: a byte table per side (p's stones -> 0x01 bytes, q's -> 0xFF; p and q
  // are disjoint, so the byte sums never carry)
  void to_board(const Key& k, int8_t* s) const {
    struct Tables {
      uint64_t one[256], neg[256];
      Tables() {
        for (int b = 0; b < 256; ++b) {
          one[b] = neg[b] = 0;
          for (int j = 0; j < 8; ++j)
            if ((b >> j) & 1) {
              one[b] |= 0x01ull << (8 * j);
              neg[b] |= 0xFFull << (8 * j);
            }
        }
      }
    };
    static const Tables T;
    int i = 0;
    for (; i + 8 <= cells; i += 8) {
      const uint64_t v = T.one[(k.p >> i) & 255] + T.neg[(k.q >> i) & 255];
      std::memcpy(s + i, &v, 8);
    }
    for (; i < cells; ++i)
      s[i] = (int8_t)(((k.p >> i) & 1) ? 1 : (((k.q >> i) & 1) ? -1 : 0));
  }
};

// ----------------------------------------------------------------------------- numpy RandomState
// np.random.RandomState(seed) (legacy MT19937: init_genrand seeding, 53-bit doubles from two
// draws, masked-rejection bounded ints) and the two RandomState.choice forms the episode uses
// (Coach.py:62 `choice(len(pi), p=pi)`, MCTS.py:41 `choice(bestAs)`), draw for draw.
struct MT19937 {
  uint32_t s[624];
  int i = 624;
  void seed(uint32_t x) {
    s[0] = x;
    for (int k = 1; k < 624; ++k) s[k] = 1812433253u * (s[k - 1] ^ (s[k - 1] >> 30)) + (uint32_t)k;
    i = 624;
  }
  void twist() {
    for (int k = 0; k < 624; ++k) {
      const uint32_t y = (s[k] & 0x80000000u) | (s[(k + 1) % 624] & 0x7fffffffu);
      s[k] = s[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    i = 0;
  }
  uint32_t next() {
    if (i >= 624) twist();
    uint32_t y = s[i++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  double next_double() {                        // random_sample()
    const uint32_t a = next() >> 5, b = next() >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
  int64_t randint(int64_t n) {                  // randint(0, n), legacy masked rejection
    const uint64_t rng = (uint64_t)(n - 1);
    if (rng == 0) return 0;
    uint64_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
    uint32_t v;
    while ((v = next() & (uint32_t)mask) > rng) {}
    return v;
  }
  int choice_p(const double* p, int n) {        // choice(n, p=p): cumsum / last, searchsorted right
    double cdf[130];
    cdf[0] = p[0];
    for (int k = 1; k < n; ++k) cdf[k] = cdf[k - 1] + p[k];
    const double last = cdf[n - 1];
    for (int k = 0; k < n; ++k) cdf[k] /= last;
    const double u = next_double();
    int k = 0;
    while (k < n && !(cdf[k] > u)) ++k;
    return k;
  }
};

// ----------------------------------------------------------------------------- episodes
// Coach.executeEpisode (Coach.py:27-79) as a per-slot state machine: getActionProb's searches,
// its pi and temp-0 tie-break, expand_tree's extra searches and root prediction, the move draw,
// the rules.  Every move is recorded; Python assembles the examples from the records with the
// same code as the sequential path (mcts_native.assemble_episode).
enum Phase : uint8_t { E_IDLE, E_START_MOVE, E_AP, E_EXP_CHECK, E_EXP_PRE, E_EXP_STD, E_EXP, E_MOVE,
                       E_DONE, E_ABORTED };

struct Episode {
  Phase phase = E_IDLE;
  bool harvested = true;
  MT19937 rng;
  Key board{0, 0};        // canonical board of the player to move
  int cur = 1, step = 0;
  int sims = 0, expand_by = 0, temp_threshold = 0;
  Val result{0.0, T_INT};
  // per-move records, A-strided
  std::vector<Key> boards;
  std::vector<int8_t> curs, temps;
  std::vector<int32_t> actions, counts, init_nsa, exp_nsa;
  std::vector<int8_t> init_has, exp_tag;
  std::vector<double> pi, exp_q;
  std::vector<float> std_v;
  void reset() {
    boards.clear(); curs.clear(); temps.clear(); actions.clear(); counts.clear();
    init_nsa.clear(); exp_nsa.clear(); init_has.clear(); exp_tag.clear(); pi.clear();
    exp_q.clear(); std_v.clear();
    board = {0, 0};
    cur = 1;
    step = 0;
    result = {0.0, T_INT};
  }
};

// ----------------------------------------------------------------------------- trees
// One cache line per node (alignas): a 56-byte node straddled two lines at most indices, and the
// descent's prefetch brought in only the first.
struct alignas(64) Node {
  Key key;
  Val es;            // Es[s]
  int32_t edge;      // offset / A into the edge pools; -1 until Vs[s] exists
  int32_t ns;        // Ns[s] (valid when has_ns)
  int32_t std_epoch; // standard_predictions epoch holding std_v
  float std_v;
  uint8_t has_ns, expanded;
};

// One edge (s, a): prior, typed Q, visit count, child node, valid flag -- packed so that a
// node's A edges are one contiguous run of cache lines (a descent touches them together).
struct Edge {
  double P;
  double qx;       // Q value (qtag == T_NONE: no Qsa entry yet)
  int32_t N;
  int32_t C;       // child node once known (-1): a descent follows it instead of re-deriving
                   // and hashing the next state
  uint8_t qtag;
  uint8_t V;       // valid move
};

// 64-byte aligned storage for the edge pool: a node's A edges (8 x 32 B for Connect4 7x7) then
// occupy whole cache lines instead of one more, straddled, line per node.
template <class T>
struct Aligned64 {
  using value_type = T;
  Aligned64() = default;
  template <class U>
  Aligned64(const Aligned64<U>&) {}
  T* allocate(size_t n) {
    return static_cast<T*>(::operator new(n * sizeof(T), std::align_val_t(64)));
  }
  void deallocate(T* p, size_t) { ::operator delete(p, std::align_val_t(64)); }
  template <class U>
  bool operator==(const Aligned64<U>&) const { return true; }
  template <class U>
  bool operator!=(const Aligned64<U>&) const { return false; }
};

// Transposition table slot: the key is stored beside the node id, so a probe compares keys in
// the slot's own cache line instead of loading the node (a second dependent miss per probe).
struct HSlot {
  Key key;
  int32_t id;      // -1 = empty
  int32_t pad;
};

struct Tree {
  std::vector<Node> nodes;
  std::vector<HSlot> table;     // open addressing
  uint64_t mask = 0;
  std::vector<Edge, Aligned64<Edge>> EP;   // edge pool, A entries per allocated node
  int32_t edges = 0;
  int32_t epoch = 1;
  // search state
  Key root{0, 0};
  int32_t root_id = -1;         // node of `root` once looked up (set_root invalidates it)
  int remaining = 0;
  int pending_leaf = -1;                      // node waiting for the network
  std::vector<std::pair<int32_t, int32_t>> path;   // (node, its chosen edge's index in EP)
  int64_t nsa_total = 0, ps_count = 0;
  int64_t cache_hits = 0;                     // leaves expanded from az_mcts_cache_put rows
  bool pending_std = false;                   // episode mode: waiting for the root's predict
  Episode ep;

  void clear() {
    nodes.clear();
    table.assign(1024, HSlot{{0, 0}, -1, 0});
    mask = 1023;
    EP.clear();
    edges = 0;
    epoch = 1;
    remaining = 0;
    pending_leaf = -1;
    pending_std = false;
    root_id = -1;
    path.clear();
    nsa_total = ps_count = 0;
  }

  void set_root(const Key& k) {
    root = k;
    root_id = -1;
  }

  // capacity for `hint` nodes up front (an episode's tree: az_mcts_episode_begin): growing the
  // node and edge pools by doubling copied them ~3 times per episode and returned the old blocks
  // to the OS (page faults, TLB shootdowns across the engine's threads); reserved pages are not
  // touched until used.  The table starts at the size `hint` nodes fill to load 1/2 or less.
  void reserve(int32_t hint, int A) {
    nodes.reserve((size_t)hint);
    EP.reserve((size_t)hint * A);
    size_t tsz = 1024;
    while (tsz * 2 <= (size_t)hint * 2) tsz *= 2;
    if (tsz > table.size()) {
      table.assign(tsz, HSlot{{0, 0}, -1, 0});
      mask = tsz - 1;
    }
  }

  int32_t find(const Key& k) const {
    if (table.empty()) return -1;
    for (uint64_t h = khash(k) & mask;; h = (h + 1) & mask) {
      const HSlot& e = table[h];
      if (e.id < 0) return -1;
      if (e.key == k) return e.id;
    }
  }

  // the slot a lookup of k starts at (run_window prefetches it a step ahead)
  const HSlot* home(const Key& k) const { return table.empty() ? nullptr : &table[khash(k) & mask]; }

  void grow() {
    std::vector<HSlot> t(table.size() * 2, HSlot{{0, 0}, -1, 0});
    uint64_t m = t.size() - 1;
    for (int32_t i = 0; i < (int32_t)nodes.size(); ++i) {
      uint64_t h = khash(nodes[i].key) & m;
      while (t[h].id >= 0) h = (h + 1) & m;
      t[h] = HSlot{nodes[i].key, i, 0};
    }
    table.swap(t);
    mask = m;
  }

  int32_t find_or_add(const Key& k, const Rules& R) {
    if (table.empty()) clear();
    uint64_t h = khash(k) & mask;
    for (;; h = (h + 1) & mask) {
      const HSlot& e = table[h];
      if (e.id < 0) break;
      if (e.key == k) return e.id;
    }
    Node nd;
    nd.key = k;
    nd.es = R.ended(k);                          // Es[s] on first visit (MCTS.py:152-153)
    nd.edge = -1;
    nd.ns = 0;
    nd.std_epoch = 0;
    nd.std_v = 0.f;
    nd.has_ns = nd.expanded = 0;
    int32_t id = (int32_t)nodes.size();
    nodes.push_back(nd);
    // the node's edge block is block `id` of the pool, reserved now (alloc_edges fills it): a
    // descent knows where a child's edges live as soon as it knows the child, so it requests
    // the node and its edge lines together (one dependent miss per tree level, not two)
    EP.resize((size_t)(id + 1) * R.A, Edge{0.0, 0.0, 0, -1, T_NONE, 0});
    table[h] = HSlot{k, id, 0};
    if ((uint64_t)nodes.size() * 2 > table.size()) grow();
    return id;
  }

  void alloc_edges(int32_t id, const Rules& R) {
    Node& nd = nodes[id];
    if (nd.edge >= 0) return;
    nd.edge = id;                                // the block find_or_add reserved
    edges += 1;
    size_t A = R.A;
    uint8_t v[kMaxA];
    R.valids(nd.key, v);
    Edge* e = &EP[(size_t)nd.edge * A];
    for (size_t a = 0; a < A; ++a) e[a].V = v[a];
  }
};

}  // namespace

// Network rows computed ahead of the search (az_mcts_cache_put): board key -> [pi, v, gpi, gv].
// Read-only while searches run, so the slots of a parallel collect may share it.
struct RowCache {
  std::vector<Key> keys;
  std::vector<int32_t> table;                   // open addressing, -1 = empty
  std::vector<float> rows;                      // stride 2A + 2
  int stride = 0;
  const float* find(const Key& k) const {
    if (keys.empty()) return nullptr;
    const uint64_t mask = table.size() - 1;
    for (uint64_t h = khash(k) & mask;; h = (h + 1) & mask) {
      const int32_t i = table[h];
      if (i < 0) return nullptr;
      if (keys[i] == k) return &rows[(size_t)i * stride];
    }
  }
  void rehash(size_t cap) {
    table.assign(cap, -1);
    for (int32_t i = 0; i < (int32_t)keys.size(); ++i) {
      uint64_t h = khash(keys[i]) & (cap - 1);
      while (table[h] >= 0) h = (h + 1) & (cap - 1);
      table[h] = i;
    }
  }
  float* insert(const Key& k) {               // the row of k (existing rows are overwritten)
    if (table.empty()) table.assign(1024, -1);
    const uint64_t mask = table.size() - 1;
    uint64_t h = khash(k) & mask;
    for (;; h = (h + 1) & mask) {
      const int32_t i = table[h];
      if (i < 0) break;
      if (keys[i] == k) return &rows[(size_t)i * stride];
    }
    const int32_t id = (int32_t)keys.size();
    keys.push_back(k);
    rows.resize(rows.size() + stride);
    table[h] = id;
    if (keys.size() * 2 > table.size()) rehash(table.size() * 2);
    return &rows[(size_t)id * stride];
  }
  void clear() {
    keys.clear();
    table.clear();
    rows.clear();
  }
};

struct az_mcts {
  Rules R;
  double cpuct = 1.0;
  int use_gnn = 0;
  std::vector<Tree> trees;
  std::vector<int32_t> last_order;             // slots of the last collect, in output order
  std::vector<int32_t> row_of;                 // feed_collect: slot -> row of the fed batch
  std::vector<int8_t> leafbuf;
  int threads = 1;                             // host threads of the last collect (feed too)
  RowCache cache;
  int spec_slot = -1;                          // az_mcts_collect_spec: slot of the pending leaf
  std::vector<Key> spec_keys;                  // ... and the children that ride along
};

namespace {

bool slot_ok(const az_mcts* m, int s) { return m && s >= 0 && s < (int)m->trees.size(); }

// UCB selection (MCTS.py:202-218); -1 when no valid action.
int select_action(const az_mcts* m, const Tree& t, const Node& nd) {
  const int A = m->R.A;
  const size_t o = (size_t)nd.edge * A;
  const double sq = std::sqrt((double)nd.ns);
  const double sq_eps = std::sqrt((double)nd.ns + 1e-8);
  double best = -INFINITY;
  int ba = -1;
  for (int a = 0; a < A; ++a) {
    const Edge& ed = t.EP[o + a];
    if (!ed.V) continue;
    double u;
    if (ed.qtag != T_NONE)
      u = ed.qx + m->cpuct * ed.P * sq / (double)(1 + ed.N);
    else
      u = m->cpuct * ed.P * sq_eps;
    if (u > best) {
      best = u;
      ba = a;
    }
  }
  return ba;
}

void backup(az_mcts* m, Tree& t, Val v) {
  (void)m;
  for (size_t i = t.path.size(); i-- > 0;) {
    Node& nd = t.nodes[t.path[i].first];
    Edge& ed = t.EP[(size_t)t.path[i].second];
    if (ed.qtag != T_NONE) {
      const Val q = div_n(add(mul_n(ed.N, Val{ed.qx, ed.qtag}), v), (long)ed.N + 1);
      ed.qx = q.x;
      ed.qtag = q.tag;
      ed.N += 1;
    } else {
      ed.qx = v.x;
      ed.qtag = v.tag;
      ed.N = 1;
    }
    t.nsa_total += 1;
    nd.ns += 1;
    v = vneg(v);                                 // two-player games (MCTS.py:236-240)
  }
  t.path.clear();
}

void expand(az_mcts* m, Tree& t, const float* pi, float v_std, const float* gpi, float gv,
            bool failed);

// Searches of many slots, interleaved one tree level at a time over a window of kWin slots (the
// slots' trees are independent, so each tree sees exactly the sequence of searches and episode
// steps it would see alone).  A descent is a chain of dependent cache misses -- a node and its
// edge block, then the child -- so one slot at a time leaves the core waiting on DRAM; here every
// window slot's next node and edge lines are requested a pass ahead and the other slots' steps
// run while they arrive.  A slot leaves the window when it waits on a new leaf (or the network,
// or has nothing left) and the next slot of the source takes its place at once: the window
// stays full (with fixed groups of 8, descents of unequal depth left ~2.6 slots live per pass
// on average).  A new leaf with a cached row (az_mcts_cache_put / az_mcts_feed_spec) is
// expanded on the spot.
constexpr int kWin = 8;

inline bool searching(const Tree& t) { return t.remaining > 0 && t.pending_leaf < 0; }

inline void prefetch_node(const Tree& t, int32_t id) { __builtin_prefetch(&t.nodes[id]); }

// a node's line and its edge block's lines (block id: find_or_add), requested together
inline void prefetch_node_edges(const Tree& t, int32_t id, int A) {
  __builtin_prefetch(&t.nodes[id]);
  const char* p = reinterpret_cast<const char*>(&t.EP[(size_t)id * A]);
  const size_t bytes = sizeof(Edge) * (size_t)A;
  for (size_t o = 0; o < bytes; o += 64) __builtin_prefetch(p + o);
}

int drive_episode(az_mcts* m, Tree& t);

// does slot t have a descent to run now?  drive: episode-mode slots first advance their episode
// (drive_episode: move bookkeeping, the next move's searches) until they need a descent, wait on
// the network or are done
inline bool has_descent(az_mcts* m, Tree& t, bool drive) {
  if (!drive) return searching(t);
  if (t.pending_leaf >= 0 || t.pending_std) return false;
  return (t.ep.phase != E_IDLE ? drive_episode(m, t) : (searching(t) ? 2 : 0)) == 2;
}

// next(): the source's next slot (nullptr when exhausted)
template <class Next>
void run_window(az_mcts* m, Next next, bool drive) {
  enum : uint8_t { START, NODE, SELECT, LOOKUP };
  const int A = m->R.A;
  Tree* ts[kWin];
  int32_t id[kWin];
  Key nkey[kWin];          // LOOKUP: the child state whose table slot was prefetched
  int32_t eidx[kWin];      // ... and the edge that will point at it
  uint8_t ph[kWin];
  auto admit = [&](int i) {                     // window place i <- the source's next slot
    while (Tree* t = next())
      if (has_descent(m, *t, drive)) {
        ts[i] = t;
        ph[i] = START;
        return true;
      }
    return false;
  };
  int n = 0;
  while (n < kWin && admit(n)) ++n;
  // slot i has no descent in progress: its next one, else the next slot (false: none left)
  auto retire = [&](int i) {
    if (has_descent(m, *ts[i], drive)) {
      ph[i] = START;
      return true;
    }
    return admit(i);
  };
  while (n > 0) {
    for (int i = 0; i < n;) {
      Tree& t = *ts[i];
      bool keep = true;
      switch (ph[i]) {
        case START:
          t.path.clear();
          if (t.root_id < 0) t.root_id = t.find_or_add(t.root, m->R);
          id[i] = t.root_id;
          prefetch_node_edges(t, id[i], A);
          ph[i] = NODE;
          break;
        case NODE: {
          const Node& nd = t.nodes[id[i]];
          if (nd.es.x != 0.0) {                  // terminal (MCTS.py:152-157)
            backup(m, t, nd.es);
            t.remaining -= 1;
            keep = retire(i);
          } else if (!nd.expanded) {             // new leaf: Vs, then the network
            t.alloc_edges(id[i], m->R);
            t.pending_leaf = id[i];
            const float* row = m->cache.find(t.nodes[id[i]].key);
            if (row) {
              // a row computed ahead (bit-identical to this leaf's own evaluation): expand now
              expand(m, t, row, row[A], m->use_gnn ? row + A + 1 : nullptr,
                     m->use_gnn ? row[2 * A + 1] : 0.f, false);
              t.cache_hits += 1;
            }
            keep = retire(i);
          } else {                               // its edges were requested with it:
            ph[i] = SELECT;                      // select in this same pass
            goto select;
          }
          break;
        }
        case SELECT:
        select: {
          const Node& nd = t.nodes[id[i]];
          const int a = select_action(m, t, nd);
          if (a < 0) {                           // MCTS.py:220-221
            backup(m, t, vint(0));
            t.remaining -= 1;
            keep = retire(i);
            break;
          }
          const size_t e = (size_t)nd.edge * A + a;
          t.path.emplace_back(id[i], (int32_t)e);
          const int32_t child = t.EP[e].C;
          if (child < 0) {                       // first visit of this edge: look the child state
            m->R.next(nd.key, a, &nkey[i]);      // up next pass, its table slot prefetched now
            eidx[i] = (int32_t)e;
            if (const HSlot* h = t.home(nkey[i])) __builtin_prefetch(h);
            ph[i] = LOOKUP;
            break;
          }
          id[i] = child;
          prefetch_node_edges(t, child, A);
          ph[i] = NODE;
          break;
        }
        default: {                               // LOOKUP
          const int32_t child = t.find_or_add(nkey[i], m->R);   // may grow t.nodes
          t.EP[(size_t)eidx[i]].C = child;
          id[i] = child;
          prefetch_node_edges(t, child, A);
          ph[i] = NODE;
          break;
        }
      }
      if (keep) {
        ++i;
      } else {                                   // the window shrinks: the last place moves here
        --n;
        ts[i] = ts[n];
        id[i] = id[n];
        nkey[i] = nkey[n];
        eidx[i] = eidx[n];
        ph[i] = ph[n];
      }
    }
  }
}

// Run searches of one slot until it waits on a leaf (returns 1) or has none left (0).
int advance(az_mcts* m, Tree& t) {
  Tree* one = &t;
  run_window(m, [&]() { Tree* r = one; one = nullptr; return r; }, false);
  return t.pending_leaf >= 0 ? 1 : 0;
}

// drive_episode's view of a slot's queued searches: 1 = waiting on a leaf, 2 = descents to run
// (run_window), 0 = none left
inline int search_state(const Tree& t) {
  if (t.pending_leaf >= 0) return 1;
  return t.remaining > 0 ? 2 : 0;
}

// Expand the pending leaf with one network row and back its value up (MCTS.py:162-200).
void expand(az_mcts* m, Tree& t, const float* pi, float v_std, const float* gpi, float gv,
            bool failed) {
  const int A = m->R.A;
  Node& nd = t.nodes[t.pending_leaf];
  Edge* ed = &t.EP[(size_t)nd.edge * A];
  double P[kMaxA];
  uint8_t V[kMaxA];
  for (int a = 0; a < A; ++a) V[a] = ed[a].V;
  Val v;
  auto uniform = [&]() {
    long cnt = 0;
    for (int a = 0; a < A; ++a) cnt += V[a];
    for (int a = 0; a < A; ++a) P[a] = (double)V[a] / (double)cnt;
  };
  if (failed) {
    uniform();
    v = vint(0);
  } else {
    nd.std_v = v_std;                            // standard_predictions[s] = (pi, v)
    nd.std_epoch = t.epoch;
    const float* src = m->use_gnn ? gpi : pi;
    for (int a = 0; a < A; ++a) P[a] = (double)src[a] * (double)V[a];
    double s = pairwise(P, A);
    if (s > 0) {
      for (int a = 0; a < A; ++a) P[a] /= s;
    } else {
      uniform();                                 // "All valid moves were masked"
    }
    v = {(double)(m->use_gnn ? gv : v_std), T_F32};
  }
  for (int a = 0; a < A; ++a) ed[a].P = P[a];
  nd.expanded = 1;
  nd.has_ns = 1;
  nd.ns = 0;
  t.ps_count += 1;
  t.pending_leaf = -1;
  backup(m, t, v);
  t.remaining -= 1;
}

// Root statistics into A-strided record arrays.
void root_snapshot(const az_mcts* m, const Tree& t, const Key& root, int32_t* nsa, double* q,
                   int8_t* tag) {
  const int A = m->R.A;
  for (int a = 0; a < A; ++a) {
    nsa[a] = 0;
    if (q) q[a] = 0.0;
    tag[a] = AZM_TAG_NONE;
  }
  const int32_t id = t.find(root);
  if (id < 0 || t.nodes[id].edge < 0) return;
  const size_t o = (size_t)t.nodes[id].edge * A;
  for (int a = 0; a < A; ++a) {
    const Edge& ed = t.EP[o + a];
    if (ed.qtag == T_NONE) continue;
    const Val v{ed.qx, ed.qtag};
    nsa[a] = ed.N;
    if (q) q[a] = v.x;
    tag[a] = v.tag == T_INT ? AZM_TAG_INT : (v.tag == T_F64 ? AZM_TAG_FLOAT : AZM_TAG_F32);
  }
}

// getActionProb's tail (MCTS.py:36-58): counts -> pi, temp-0 tie-break on the slot's RNG.
void finish_action_prob(const az_mcts* m, Tree& t) {
  Episode& E = t.ep;
  const int A = m->R.A;
  const size_t mv = E.curs.size() - 1;
  int32_t* cnt = &E.counts[mv * A];
  std::vector<int8_t> tag(A);
  root_snapshot(m, t, E.board, cnt, nullptr, tag.data());
  double* pi = &E.pi[mv * A];
  if (E.temps[mv] == 0) {
    int32_t mx = cnt[0];
    for (int a = 1; a < A; ++a) mx = cnt[a] > mx ? cnt[a] : mx;
    int best[130], nb = 0;
    for (int a = 0; a < A; ++a)
      if (cnt[a] == mx) best[nb++] = a;
    const int a = best[E.rng.randint(nb)];
    for (int k = 0; k < A; ++k) pi[k] = k == a ? 1.0 : 0.0;
  } else {
    double total = 0.0;                         // float(sum(...)), sequential
    for (int a = 0; a < A; ++a) total += (double)cnt[a] + 1e-8;
    for (int a = 0; a < A; ++a) pi[a] = ((double)cnt[a] + 1e-8) / total;
  }
}

// Advance one episode-mode slot until it waits on the network (1) or is done (0).
int drive_episode(az_mcts* m, Tree& t) {
  Episode& E = t.ep;
  const int A = m->R.A;
  for (;;) {
    switch (E.phase) {
      case E_START_MOVE: {
        E.step += 1;
        t.epoch += 1;                           // getActionProb resets the predictions
        E.boards.push_back(E.board);
        E.curs.push_back((int8_t)E.cur);
        E.temps.push_back((int8_t)(E.step < E.temp_threshold ? 1 : 0));
        E.actions.push_back(-1);
        E.counts.resize(E.counts.size() + A, 0);
        E.pi.resize(E.pi.size() + A, 0.0);
        E.init_nsa.resize(E.init_nsa.size() + A, 0);
        E.init_has.resize(E.init_has.size() + A, (int8_t)AZM_TAG_NONE);
        E.exp_nsa.resize(E.exp_nsa.size() + A, 0);
        E.exp_q.resize(E.exp_q.size() + A, 0.0);
        E.exp_tag.resize(E.exp_tag.size() + A, (int8_t)AZM_TAG_NONE);
        E.std_v.push_back(0.f);
        t.set_root(E.board);
        t.remaining = E.sims;
        E.phase = E_AP;
        break;
      }
      case E_AP:
        if (const int r = search_state(t)) return r;
        finish_action_prob(m, t);
        E.phase = m->use_gnn ? E_EXP_CHECK : E_MOVE;
        break;
      case E_EXP_CHECK: {                       // expand_tree (MCTS.py:60-149)
        const size_t mv = E.curs.size() - 1;
        root_snapshot(m, t, E.board, &E.init_nsa[mv * A], nullptr, &E.init_has[mv * A]);
        bool any = false;
        for (int a = 0; a < A; ++a) any |= E.init_has[mv * A + a] != AZM_TAG_NONE;
        if (any) {
          E.phase = E_EXP_STD;
        } else {
          t.set_root(E.board);
          t.remaining = E.sims;
          E.phase = E_EXP_PRE;
        }
        break;
      }
      case E_EXP_PRE: {
        if (const int r = search_state(t)) return r;
        const size_t mv = E.curs.size() - 1;
        root_snapshot(m, t, E.board, &E.init_nsa[mv * A], nullptr, &E.init_has[mv * A]);
        E.phase = E_EXP_STD;
        break;
      }
      case E_EXP_STD: {
        const int32_t id = t.find(E.board);
        if (id >= 0 && t.nodes[id].std_epoch == t.epoch) {
          E.std_v.back() = t.nodes[id].std_v;
          t.set_root(E.board);
          t.remaining = E.expand_by;
          E.phase = E_EXP;
        } else {
          t.pending_std = true;                 // root predict (served by the next batch)
          return 1;
        }
        break;
      }
      case E_EXP: {
        if (const int r = search_state(t)) return r;
        const size_t mv = E.curs.size() - 1;
        root_snapshot(m, t, E.board, &E.exp_nsa[mv * A], &E.exp_q[mv * A], &E.exp_tag[mv * A]);
        E.phase = E_MOVE;
        break;
      }
      case E_MOVE: {                            // Coach.py:62-79
        const size_t mv = E.curs.size() - 1;
        const int a = E.rng.choice_p(&E.pi[mv * A], A);
        E.actions[mv] = a;
        Key nk;
        m->R.next(E.board, a, &nk);
        E.board = nk;
        E.cur = -E.cur;
        const Val r = m->R.ended(nk);
        if (r.x != 0.0) {
          E.result = r;
          E.phase = E_DONE;
          E.harvested = false;
          return 0;
        }
        E.phase = E_START_MOVE;
        break;
      }
      default:
        return 0;
    }
  }
}

}  // namespace

extern "C" {

const char* az_mcts_last_error(void) { return g_err.c_str(); }

az_mcts* az_mcts_create(int game, int n, int slots, double cpuct, int use_gnn) {
  if (slots < 1) {
    fail(AZM_EINVAL, "az_mcts_create: slots must be >= 1");
    return nullptr;
  }
  az_mcts* m = new az_mcts();
  if (!m->R.init(game, n)) {
    delete m;
    fail(AZM_EINVAL, "az_mcts_create: unsupported game / board size (n*n must be <= 64)");
    return nullptr;
  }
  m->cpuct = cpuct;
  m->use_gnn = use_gnn;
  m->trees.resize(slots);
  for (auto& t : m->trees) t.clear();
  m->leafbuf.resize((size_t)slots * m->R.cells);
  return m;
}

void az_mcts_destroy(az_mcts* m) { delete m; }

int az_mcts_action_size(const az_mcts* m) { return m ? m->R.A : AZM_EINVAL; }

int az_mcts_reset(az_mcts* m, int slot) {
  if (!slot_ok(m, slot)) return fail(AZM_EINVAL, "az_mcts_reset: bad slot");
  m->trees[slot].clear();
  m->trees[slot].ep.phase = E_IDLE;
  m->trees[slot].ep.harvested = true;
  return AZM_OK;
}

int az_mcts_episode_begin(az_mcts* m, int slot, uint32_t seed, int sims, int expand_by,
                          int temp_threshold) {
  if (!slot_ok(m, slot) || sims < 0 || expand_by < 0)
    return fail(AZM_EINVAL, "az_mcts_episode_begin: bad args");
  Tree& t = m->trees[slot];
  t.clear();
  // an episode's tree holds ~sims x (moves ~ cells) / 1.4 nodes (Connect4 7x7 at 100 sims: 3,408
  // on average, 4,155 at most, tools/native/mcts_prof.cpp): room for sims x cells
  t.reserve((int32_t)std::min<int64_t>((int64_t)std::max(sims, 1) * m->R.cells, 32768), m->R.A);
  Episode& E = t.ep;
  E.reset();
  E.rng.seed(seed);
  E.sims = sims;
  E.expand_by = expand_by;
  E.temp_threshold = temp_threshold;
  E.harvested = true;
  E.phase = E_START_MOVE;
  return AZM_OK;
}

int az_mcts_episode_finished(az_mcts* m, int32_t* slots, int cap) {
  if (!m || !slots) return fail(AZM_EINVAL, "az_mcts_episode_finished: bad args");
  int n = 0;
  for (int s = 0; s < (int)m->trees.size() && n < cap; ++s) {
    Episode& E = m->trees[s].ep;
    if (E.phase == E_DONE && !E.harvested) {
      E.harvested = true;
      slots[n++] = s;
    }
  }
  return n;
}

int az_mcts_episode_moves(const az_mcts* m, int slot) {
  if (!slot_ok(m, slot)) return fail(AZM_EINVAL, "az_mcts_episode_moves: bad slot");
  return (int)m->trees[slot].ep.curs.size();
}

int az_mcts_episode_record(const az_mcts* m, int slot, int8_t* boards, int8_t* curs,
                           int8_t* temps, int32_t* actions, double* pi, int32_t* init_nsa,
                           int8_t* init_has, float* std_v, int32_t* exp_nsa, double* exp_q,
                           int8_t* exp_tag, int* result_tag, double* result) {
  if (!slot_ok(m, slot)) return fail(AZM_EINVAL, "az_mcts_episode_record: bad slot");
  const Episode& E = m->trees[slot].ep;
  const int A = m->R.A, C = m->R.cells;
  const size_t n = E.curs.size();
  for (size_t i = 0; i < n; ++i) m->R.to_board(E.boards[i], boards + i * C);
  std::memcpy(curs, E.curs.data(), n);
  std::memcpy(temps, E.temps.data(), n);
  std::memcpy(actions, E.actions.data(), n * 4);
  std::memcpy(pi, E.pi.data(), n * A * 8);
  std::memcpy(init_nsa, E.init_nsa.data(), n * A * 4);
  std::memcpy(init_has, E.init_has.data(), n * A);
  std::memcpy(std_v, E.std_v.data(), n * 4);
  std::memcpy(exp_nsa, E.exp_nsa.data(), n * A * 4);
  std::memcpy(exp_q, E.exp_q.data(), n * A * 8);
  std::memcpy(exp_tag, E.exp_tag.data(), n * A);
  *result_tag = E.result.tag == T_INT ? AZM_TAG_INT : AZM_TAG_FLOAT;
  *result = E.result.x;
  return AZM_OK;
}

int az_mcts_episode_targets(const az_mcts* m, int slot, double* init_policy, double* exp_policy,
                            int8_t* exp_value_tag, double* exp_value) {
  if (!slot_ok(m, slot) || !init_policy || !exp_policy || !exp_value_tag || !exp_value)
    return fail(AZM_EINVAL, "az_mcts_episode_targets: bad args");
  const Episode& E = m->trees[slot].ep;
  const int A = m->R.A;
  std::vector<uint8_t> valid(A);
  for (size_t i = 0; i < E.curs.size(); ++i) {
    double* ip = init_policy + i * A;
    double* xp = exp_policy + i * A;
    const int32_t* inn = &E.init_nsa[i * A];
    const int8_t* ih = &E.init_has[i * A];
    const int32_t* xn = &E.exp_nsa[i * A];
    const int8_t* xt = &E.exp_tag[i * A];
    const double* xq = &E.exp_q[i * A];
    // counts are integers: their float64 sums are exact in any order (np.sum's pairwise too)
    double isum = 0.0;
    for (int a = 0; a < A; ++a) {
      ip[a] = ih[a] != AZM_TAG_NONE ? (double)inn[a] : 0.0;
      isum += ip[a];
    }
    if (isum > 0) {
      for (int a = 0; a < A; ++a) ip[a] /= isum;
    } else {                                   // valids / np.sum(valids)
      m->R.valids(E.boards[i], valid.data());
      double vs = 0.0;
      for (int a = 0; a < A; ++a) vs += valid[a];
      for (int a = 0; a < A; ++a) ip[a] = (double)valid[a] / vs;
    }
    double esum = 0.0;
    for (int a = 0; a < A; ++a) {
      xp[a] = xt[a] != AZM_TAG_NONE ? (double)xn[a] : 0.0;
      esum += xp[a];
    }
    if (esum > 0) {
      for (int a = 0; a < A; ++a) xp[a] /= esum;
    } else {
      for (int a = 0; a < A; ++a) xp[a] = ip[a];
    }
    // expanded_value = sum(typed Q * N) / sum(N) over visited edges, else the root's value
    Val ev = vint(0);
    long cnt = 0;
    for (int a = 0; a < A; ++a) {
      if (xt[a] == AZM_TAG_NONE || xn[a] <= 0) continue;
      const Val q{xq[a], xt[a] == AZM_TAG_INT ? T_INT : (xt[a] == AZM_TAG_FLOAT ? T_F64 : T_F32)};
      ev = add(ev, mul_n(xn[a], q));
      cnt += xn[a];
    }
    if (cnt > 0) {
      ev = div_n(ev, cnt);
    } else {
      ev = {(double)E.std_v[i], T_F32};
    }
    exp_value_tag[i] = ev.tag == T_INT ? AZM_TAG_INT : (ev.tag == T_F64 ? AZM_TAG_FLOAT : AZM_TAG_F32);
    exp_value[i] = ev.x;
  }
  return AZM_OK;
}

int az_mcts_episodes_moves(const az_mcts* m, const int32_t* slots, int n, int32_t* moves) {
  if (!m || (n > 0 && (!slots || !moves)) || n < 0)
    return fail(AZM_EINVAL, "az_mcts_episodes_moves: bad args");
  for (int i = 0; i < n; ++i) {
    if (!slot_ok(m, slots[i])) return fail(AZM_EINVAL, "az_mcts_episodes_moves: bad slot");
    moves[i] = (int32_t)m->trees[slots[i]].ep.curs.size();
  }
  return AZM_OK;
}

int az_mcts_episode_records(const az_mcts* m, const int32_t* slots, int n, int8_t* boards,
                            int8_t* curs, int8_t* temps, int32_t* actions, double* pi,
                            int32_t* init_nsa, int8_t* init_has, float* std_v, int32_t* exp_nsa,
                            double* exp_q, int8_t* exp_tag, int* result_tags, double* results,
                            double* init_policy, double* exp_policy, int8_t* exp_value_tag,
                            double* exp_value) {
  if (!m || n < 0 || (n > 0 && !slots)) return fail(AZM_EINVAL, "az_mcts_episode_records: bad args");
  const bool tg = init_policy != nullptr;
  if (tg && (!exp_policy || !exp_value_tag || !exp_value))
    return fail(AZM_EINVAL, "az_mcts_episode_records: partial target pointers");
  const size_t A = (size_t)m->R.A, C = (size_t)m->R.cells;
  size_t o = 0;                                 // first move of episode i in the outputs
  for (int i = 0; i < n; ++i) {
    const int s = slots[i];
    if (int rc = az_mcts_episode_record(m, s, boards + o * C, curs + o, temps + o, actions + o,
                                        pi + o * A, init_nsa + o * A, init_has + o * A, std_v + o,
                                        exp_nsa + o * A, exp_q + o * A, exp_tag + o * A,
                                        result_tags + i, results + i))
      return rc;
    if (tg) {
      if (int rc = az_mcts_episode_targets(m, s, init_policy + o * A, exp_policy + o * A,
                                           exp_value_tag + o, exp_value + o))
        return rc;
    }
    o += m->trees[s].ep.curs.size();
  }
  return AZM_OK;
}

int az_rng_test(uint32_t seed, int op, int n, const double* p, int np_, int64_t* out) {
  // differential-test hook: op 0 = n x next uint32, 1 = n x randint(np_), 2 = n x choice(np_, p)
  MT19937 r;
  r.seed(seed);
  for (int i = 0; i < n; ++i) {
    if (op == 0) out[i] = r.next();
    else if (op == 1) out[i] = r.randint(np_);
    else out[i] = r.choice_p(p, np_);
  }
  return AZM_OK;
}

int az_rng_doubles(uint32_t seed, int n, double* out) {
  MT19937 r;
  r.seed(seed);
  for (int i = 0; i < n; ++i) out[i] = r.next_double();
  return AZM_OK;
}

int az_mcts_clear_predictions(az_mcts* m, int slot) {
  if (!slot_ok(m, slot)) return fail(AZM_EINVAL, "az_mcts_clear_predictions: bad slot");
  m->trees[slot].epoch += 1;
  return AZM_OK;
}

int az_mcts_begin(az_mcts* m, int slot, const int8_t* board, int sims) {
  if (!slot_ok(m, slot) || !board || sims < 0) return fail(AZM_EINVAL, "az_mcts_begin: bad args");
  Tree& t = m->trees[slot];
  if (t.remaining > 0 || t.pending_leaf >= 0)
    return fail(AZM_ESTATE, "az_mcts_begin: slot still has searches queued");
  Key k;
  if (!m->R.from_board(board, &k)) return fail(AZM_EINVAL, "az_mcts_begin: cells must be -1/0/1");
  t.set_root(k);
  t.remaining = sims;
  return AZM_OK;
}

int az_mcts_remaining(const az_mcts* m, int slot) {
  if (!slot_ok(m, slot)) return fail(AZM_EINVAL, "az_mcts_remaining: bad slot");
  return m->trees[slot].remaining;
}

int az_mcts_abandon(az_mcts* m, int slot) {
  if (!slot_ok(m, slot)) return fail(AZM_EINVAL, "az_mcts_abandon: bad slot");
  Tree& t = m->trees[slot];
  if (t.pending_leaf >= 0) return fail(AZM_ESTATE, "az_mcts_abandon: a leaf waits for its feed");
  t.remaining = 0;
  return AZM_OK;
}

int az_mcts_remaining_all(const az_mcts* m, int32_t* out) {
  if (!m || !out) return fail(AZM_EINVAL, "az_mcts_remaining_all: bad args");
  for (size_t s = 0; s < m->trees.size(); ++s) out[s] = m->trees[s].remaining;
  return AZM_OK;
}

}  // extern "C"

namespace {

// One network row for a slot's pending request (az_mcts_feed's body): expand_tree's root
// predict takes v only; a leaf is expanded and its value backed up.  failed = the reference's
// uniform priors / v = 0 (MCTS.py:195-200), or an aborted episode for a root predict (unguarded
// in the reference, MCTS.py:108-113).  Returns 1 when the episode was aborted.
int feed_row(az_mcts* m, Tree& t, int i, const float* pi, const float* v, const float* gpi,
             const float* gv, bool failed) {
  const int A = m->R.A;
  if (t.pending_std) {
    t.pending_std = false;
    if (failed) {
      t.ep.phase = E_ABORTED;
      return 1;
    }
    Node& nd = t.nodes[t.find_or_add(t.ep.board, m->R)];
    nd.std_v = v[i];
    nd.std_epoch = t.epoch;
    return 0;
  }
  expand(m, t, failed ? nullptr : pi + (size_t)i * A, failed ? 0.f : v[i],
         (failed || !m->use_gnn) ? nullptr : gpi + (size_t)i * A,
         (failed || !m->use_gnn) ? 0.f : gv[i], failed);
  return 0;
}

struct FeedRows {        // rows of the previous collect, fed inside the next one
  const int32_t* row_of; // slot -> row index, -1 = none
  const float *pi, *v, *gpi, *gv;
};

// az_mcts_collect's body; with fr, each group of slots first takes its network rows (the feed
// and the next descents of a slot run back to back on one thread, in one parallel region).
int collect_impl(az_mcts* m, int8_t* boards, int32_t* slots, int cap, int threads,
                 const FeedRows* fr) {
  const int S = (int)m->trees.size();
  std::vector<uint8_t> has(S, 0);
  if (threads < 1) threads = 1;
  m->threads = threads;
  // chunks of kChunk consecutive slots per thread (dynamic): each chunk's episode state machines
  // run, kWin at a time (run_window), until every slot waits on the network or is idle
  constexpr int kChunk = 32;
  const int ngroups = (S + kChunk - 1) / kChunk;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
  for (int gi = 0; gi < ngroups; ++gi) {
    const int s0 = gi * kChunk, s1 = std::min(S, s0 + kChunk);
    if (fr) {
      // the backups touch every node and edge on each fed slot's path, last written a round ago
      // (often by another thread): their lines are requested kWin slots ahead of the feed
      auto request = [&](int s) {
        if (s >= s1 || fr->row_of[s] < 0) return;
        const Tree& t = m->trees[s];
        if (t.pending_leaf >= 0) prefetch_node_edges(t, t.pending_leaf, m->R.A);
        for (const auto& pe : t.path) {
          prefetch_node(t, pe.first);
          __builtin_prefetch(&t.EP[(size_t)pe.second]);
        }
      };
      for (int s = s0; s < s0 + kWin; ++s) request(s);
      for (int s = s0; s < s1; ++s) {
        request(s + kWin);
        if (fr->row_of[s] >= 0)
          feed_row(m, m->trees[s], fr->row_of[s], fr->pi, fr->v, fr->gpi, fr->gv, false);
      }
    }
    int nx = s0;
    run_window(m, [&]() { return nx < s1 ? &m->trees[nx++] : nullptr; }, true);
    for (int s = s0; s < s1; ++s) {
      const Tree& t = m->trees[s];
      if (t.pending_leaf >= 0) {
        has[s] = 1;
        m->R.to_board(t.nodes[t.pending_leaf].key, &m->leafbuf[(size_t)s * m->R.cells]);
      } else if (t.pending_std) {
        has[s] = 1;
        m->R.to_board(t.ep.board, &m->leafbuf[(size_t)s * m->R.cells]);
      }
    }
  }
  m->last_order.clear();
  int cnt = 0;
  for (int s = 0; s < S; ++s) {
    if (!has[s]) continue;
    if (cnt >= cap) return fail(AZM_EINVAL, "az_mcts_collect: cap smaller than the live slots");
    std::memcpy(boards + (size_t)cnt * m->R.cells, &m->leafbuf[(size_t)s * m->R.cells],
                m->R.cells);
    slots[cnt++] = s;
    m->last_order.push_back(s);
  }
  return cnt;
}

// the checks az_mcts_feed / az_mcts_feed_collect share
int check_feed(const az_mcts* m, int count, const float* pi, const float* v, const float* gpi,
               const float* gv, int failed, const char* what) {
  if (!m || count != (int)m->last_order.size())
    return fail(AZM_EINVAL, std::string(what) + ": count differs from the last collect");
  if (!failed && (!pi || !v || (m->use_gnn && (!gpi || !gv))))
    return fail(AZM_EINVAL, std::string(what) + ": missing network outputs");
  for (int i = 0; i < count; ++i) {
    const Tree& t = m->trees[m->last_order[i]];
    if (t.pending_leaf < 0 && !t.pending_std)
      return fail(AZM_ESTATE, std::string(what) + ": slot has no pending request");
  }
  return AZM_OK;
}

}  // namespace

extern "C" {

int az_mcts_collect(az_mcts* m, int8_t* boards, int32_t* slots, int cap, int threads) {
  if (!m || !boards || !slots || cap < 0) return fail(AZM_EINVAL, "az_mcts_collect: bad args");
  if (m->spec_slot >= 0)
    return fail(AZM_ESTATE, "az_mcts_collect: a collect_spec request was not fed");
  for (auto& t : m->trees)
    if (t.pending_leaf >= 0 && !m->last_order.empty())
      return fail(AZM_ESTATE, "az_mcts_collect: the previous leaves were not fed");
  return collect_impl(m, boards, slots, cap, threads, nullptr);
}

int az_mcts_feed(az_mcts* m, int count, const float* pi, const float* v, const float* gpi,
                 const float* gv, int failed) {
  if (const int rc = check_feed(m, count, pi, v, gpi, gv, failed, "az_mcts_feed")) return rc;
  // every leaf belongs to a different slot's tree: the expansions are independent
  int aborted = 0;
#pragma omp parallel for schedule(dynamic, 8) num_threads(m->threads) if (count >= 32) \
    reduction(+ : aborted)
  for (int i = 0; i < count; ++i)
    aborted += feed_row(m, m->trees[m->last_order[i]], i, pi, v, gpi, gv, failed != 0);
  m->last_order.clear();
  return aborted;
}

int az_mcts_feed_collect(az_mcts* m, int count, const float* pi, const float* v,
                         const float* gpi, const float* gv, int8_t* boards, int32_t* slots,
                         int cap, int threads) {
  if (const int rc = check_feed(m, count, pi, v, gpi, gv, 0, "az_mcts_feed_collect")) return rc;
  if (!boards || !slots || cap < 0) return fail(AZM_EINVAL, "az_mcts_feed_collect: bad args");
  if (m->spec_slot >= 0)
    return fail(AZM_ESTATE, "az_mcts_feed_collect: a collect_spec request was not fed");
  m->row_of.assign(m->trees.size(), -1);
  for (int i = 0; i < count; ++i) m->row_of[m->last_order[i]] = i;
  // the rows are applied inside the collect, so a cap the collect would overflow must fail
  // here, while nothing has changed yet (a later plain az_mcts_feed still matches last_order):
  // every slot that is fed, searching or inside an episode can hand out one leaf
  int may = 0;
  if (cap < (int)m->trees.size())          // (a cap of every slot needs no count)
    for (size_t s = 0; s < m->trees.size(); ++s) {
      const Tree& t = m->trees[s];
      may += m->row_of[s] >= 0 || t.ep.phase != E_IDLE || searching(t) || t.pending_leaf >= 0 ||
             t.pending_std;
    }
  if (cap < may)
    return fail(AZM_EINVAL, "az_mcts_feed_collect: cap " + std::to_string(cap) +
                                " smaller than the " + std::to_string(may) +
                                " slots that may hand out a leaf (nothing was fed)");
  m->last_order.clear();
  const FeedRows fr{m->row_of.data(), pi, v, gpi, gv};
  return collect_impl(m, boards, slots, cap, threads, &fr);
}

int az_mcts_cache_put(az_mcts* m, int count, const int8_t* boards, const float* pi, const float* v,
                      const float* gpi, const float* gv) {
  if (!m || count < 0 || (count > 0 && (!boards || !pi || !v)) ||
      (count > 0 && m->use_gnn && (!gpi || !gv)))
    return fail(AZM_EINVAL, "az_mcts_cache_put: bad args");
  const int A = m->R.A;
  m->cache.stride = 2 * A + 2;
  for (int i = 0; i < count; ++i) {
    Key k;
    if (!m->R.from_board(boards + (size_t)i * m->R.cells, &k))
      return fail(AZM_EINVAL, "az_mcts_cache_put: cells must be -1/0/1");
    float* r = m->cache.insert(k);
    std::memcpy(r, pi + (size_t)i * A, sizeof(float) * A);
    r[A] = v[i];
    if (m->use_gnn) {
      std::memcpy(r + A + 1, gpi + (size_t)i * A, sizeof(float) * A);
      r[2 * A + 1] = gv[i];
    } else {
      std::fill(r + A + 1, r + 2 * A + 2, 0.f);
    }
  }
  return AZM_OK;
}

int az_mcts_collect_spec(az_mcts* m, int slot, int8_t* boards, int cap) {
  if (!slot_ok(m, slot) || !boards || cap < 1)
    return fail(AZM_EINVAL, "az_mcts_collect_spec: bad args");
  if (!m->last_order.empty() || m->spec_slot >= 0)
    return fail(AZM_ESTATE, "az_mcts_collect_spec: the previous request was not fed");
  Tree& t = m->trees[slot];
  if (t.ep.phase != E_IDLE) return fail(AZM_ESTATE, "az_mcts_collect_spec: slot is in episode mode");
  if (t.pending_leaf < 0) advance(m, t);
  if (t.pending_leaf < 0) return 0;            // searches done (or none queued)
  const Rules& R = m->R;
  const Key leaf = t.nodes[t.pending_leaf].key;
  R.to_board(leaf, boards);
  int cnt = 1;
  m->spec_keys.clear();
  if (R.ended(leaf).x == 0.0) {
    uint8_t v[kMaxA];
    R.valids(leaf, v);
    Key nk;
    for (int a = 0; a < R.A && cnt < cap; ++a) {
      if (!v[a] || !R.next(leaf, a, &nk)) continue;
      if (R.ended(nk).x != 0.0) continue;       // terminal: never evaluated
      const int32_t id = t.find(nk);
      if (id >= 0 && t.nodes[id].expanded) continue;   // already has its row in the tree
      if (m->cache.find(nk)) continue;                // already speculated
      R.to_board(nk, boards + (size_t)cnt * R.cells);
      m->spec_keys.push_back(nk);
      ++cnt;
    }
  }
  m->spec_slot = slot;
  return cnt;
}

int az_mcts_feed_spec(az_mcts* m, int count, const float* pi, const float* v, const float* gpi,
                      const float* gv, int failed) {
  if (!m || m->spec_slot < 0) return fail(AZM_ESTATE, "az_mcts_feed_spec: nothing collected");
  if (count != 1 + (int)m->spec_keys.size())
    return fail(AZM_EINVAL, "az_mcts_feed_spec: count differs from the last collect_spec");
  if (!failed && (!pi || !v || (m->use_gnn && (!gpi || !gv))))
    return fail(AZM_EINVAL, "az_mcts_feed_spec: missing network outputs");
  Tree& t = m->trees[m->spec_slot];
  m->spec_slot = -1;
  const int A = m->R.A;
  if (failed) {                                 // the leaf degrades (MCTS.py:195-200), no rows kept
    expand(m, t, nullptr, 0.f, nullptr, 0.f, true);
    return AZM_OK;
  }
  m->cache.stride = 2 * A + 2;
  for (int i = 1; i < count; ++i) {
    float* r = m->cache.insert(m->spec_keys[i - 1]);
    std::memcpy(r, pi + (size_t)i * A, sizeof(float) * A);
    r[A] = v[i];
    if (m->use_gnn) {
      std::memcpy(r + A + 1, gpi + (size_t)i * A, sizeof(float) * A);
      r[2 * A + 1] = gv[i];
    } else {
      std::fill(r + A + 1, r + 2 * A + 2, 0.f);
    }
  }
  expand(m, t, pi, v[0], m->use_gnn ? gpi : nullptr, m->use_gnn ? gv[0] : 0.f, false);
  return AZM_OK;
}

int az_mcts_cache_clear(az_mcts* m) {
  if (!m) return fail(AZM_EINVAL, "az_mcts_cache_clear: bad args");
  m->cache.clear();
  return AZM_OK;
}

int az_mcts_cache_stats(const az_mcts* m, int64_t* out) {
  if (!m || !out) return fail(AZM_EINVAL, "az_mcts_cache_stats: bad args");
  int64_t hits = 0;
  for (const auto& t : m->trees) hits += t.cache_hits;
  out[0] = (int64_t)m->cache.keys.size();
  out[1] = hits;
  return AZM_OK;
}

int az_mcts_root_edges(const az_mcts* m, int slot, const int8_t* board, int32_t* nsa, double* q,
                       int8_t* qtag) {
  if (!slot_ok(m, slot) || !board) return fail(AZM_EINVAL, "az_mcts_root_edges: bad args");
  const Tree& t = m->trees[slot];
  Key k;
  if (!m->R.from_board(board, &k)) return fail(AZM_EINVAL, "az_mcts_root_edges: bad board");
  const int A = m->R.A;
  int32_t id = t.find(k);
  for (int a = 0; a < A; ++a) {
    nsa[a] = 0;
    q[a] = 0.0;
    qtag[a] = AZM_TAG_NONE;
  }
  if (id < 0 || t.nodes[id].edge < 0) return AZM_OK;
  size_t o = (size_t)t.nodes[id].edge * A;
  for (int a = 0; a < A; ++a) {
    const Edge& ed = t.EP[o + a];
    if (ed.qtag == T_NONE) continue;
    nsa[a] = ed.N;
    q[a] = ed.qx;
    qtag[a] = ed.qtag == T_INT ? AZM_TAG_INT : (ed.qtag == T_F64 ? AZM_TAG_FLOAT : AZM_TAG_F32);
  }
  return AZM_OK;
}

int az_mcts_get_std(const az_mcts* m, int slot, const int8_t* board, float* v) {
  if (!slot_ok(m, slot) || !board || !v) return fail(AZM_EINVAL, "az_mcts_get_std: bad args");
  const Tree& t = m->trees[slot];
  Key k;
  if (!m->R.from_board(board, &k)) return fail(AZM_EINVAL, "az_mcts_get_std: bad board");
  int32_t id = t.find(k);
  if (id < 0 || t.nodes[id].std_epoch != t.epoch) return 0;
  *v = t.nodes[id].std_v;
  return 1;
}

int az_mcts_set_std(az_mcts* m, int slot, const int8_t* board, float v) {
  if (!slot_ok(m, slot) || !board) return fail(AZM_EINVAL, "az_mcts_set_std: bad args");
  Tree& t = m->trees[slot];
  Key k;
  if (!m->R.from_board(board, &k)) return fail(AZM_EINVAL, "az_mcts_set_std: bad board");
  Node& nd = t.nodes[t.find_or_add(k, m->R)];
  nd.std_v = v;
  nd.std_epoch = t.epoch;
  return AZM_OK;
}

int az_mcts_tree_stats(const az_mcts* m, int slot, int64_t* out) {
  if (!slot_ok(m, slot) || !out) return fail(AZM_EINVAL, "az_mcts_tree_stats: bad args");
  const Tree& t = m->trees[slot];
  int64_t ns = 0;
  for (const auto& nd : t.nodes) ns += nd.has_ns;
  out[0] = (int64_t)t.nodes.size();
  out[1] = ns;
  out[2] = t.ps_count;
  out[3] = t.nsa_total;
  return AZM_OK;
}

int az_game_ended(int game, int n, const int8_t* board, int* tag, double* value) {
  Rules R;
  Key k;
  if (!R.init(game, n) || !R.from_board(board, &k)) return fail(AZM_EINVAL, "az_game_ended");
  Val v = R.ended(k);
  *tag = v.tag == T_INT ? AZM_TAG_INT : AZM_TAG_FLOAT;
  *value = v.x;
  return AZM_OK;
}

int az_game_valids(int game, int n, const int8_t* board, int8_t* valids) {
  Rules R;
  Key k;
  if (!R.init(game, n) || !R.from_board(board, &k)) return fail(AZM_EINVAL, "az_game_valids");
  std::vector<uint8_t> v(R.A);
  R.valids(k, v.data());
  for (int a = 0; a < R.A; ++a) valids[a] = (int8_t)v[a];
  return AZM_OK;
}

int az_game_next_canonical(int game, int n, const int8_t* board, int action, int8_t* out) {
  Rules R;
  Key k, nk;
  if (!R.init(game, n) || !R.from_board(board, &k) || action < 0 || action >= R.A)
    return fail(AZM_EINVAL, "az_game_next_canonical: bad args");
  if (!R.next(k, action, &nk)) return fail(AZM_EINVAL, "az_game_next_canonical: illegal move");
  R.to_board(nk, out);
  return AZM_OK;
}

int az_game_children(int game, int n, const int8_t* board, int cap, int8_t* out) {
  Rules R;
  Key k, nk;
  if (!R.init(game, n) || !R.from_board(board, &k) || cap < 0 || (cap > 0 && !out))
    return fail(AZM_EINVAL, "az_game_children: bad args");
  if (R.ended(k).x != 0.0) return 0;            // terminal: the search never expands it
  std::vector<uint8_t> v(R.A);
  R.valids(k, v.data());
  int cnt = 0;
  for (int a = 0; a < R.A && cnt < cap; ++a) {
    if (!v[a] || !R.next(k, a, &nk)) continue;
    if (R.ended(nk).x != 0.0) continue;         // terminal children are never evaluated
    R.to_board(nk, out + (size_t)cnt * R.cells);
    ++cnt;
  }
  return cnt;
}

double az_np_pairwise_sum(const double* a, int n) { return pairwise(a, n); }

}  // extern "C"
