// Host-only stress driver for the native MCTS engine (csrc/az_mcts.cpp), built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native_sanitize.py.  It drives
// every entry point of include/az_mcts.h the way selfplay.py / mcts_native.py do -- episode
// mode and search mode, both games at several board sizes, with and without the GNN path,
// several host threads -- with a deterministic pseudo-random "network" (priors and values a
// hash of the board, sprinkled with zeros, ties and failed batches), plus the error paths.
// Exit status 0 = every call behaved; the sanitizers abort on any memory or UB error.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/az_mcts.h"

namespace {

uint64_t mix(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  return h ^ (h >> 33);
}

// pi[A] (a probability vector, sometimes with zeros / ties) and v for a board
void fake_net(const int8_t* b, int cells, int A, uint64_t salt, float* pi, float* v) {
  uint64_t h = salt;
  for (int i = 0; i < cells; ++i) h = mix(h + (uint64_t)(b[i] + 2) * 0x9e3779b97f4a7c15ULL);
  float s = 0.f;
  for (int a = 0; a < A; ++a) {
    h = mix(h + a);
    pi[a] = (h % 7 == 0) ? 0.f : (float)((h >> 11) % 1000 + 1);
    s += pi[a];
  }
  if (h % 11 == 0) {
    for (int a = 0; a < A; ++a) pi[a] = 1.f;
    s = (float)A;
  }
  for (int a = 0; a < A; ++a) pi[a] = s > 0.f ? pi[a] / s : 0.f;
  *v = (float)((int64_t)((h >> 20) % 2001) - 1000) / 1000.f;
}

int fail(const char* what) {
  fprintf(stderr, "FAIL: %s (%s)\n", what, az_mcts_last_error());
  return 1;
}

// Whole episodes in `slots` slots until `episodes` are finished.
// fused: good batches are fed inside the next collect (az_mcts_feed_collect) and finished
// episodes exported in one az_mcts_episode_records call per round
int run_episodes(int game, int n, int slots, int use_gnn, int threads, int episodes, int sims,
                 uint64_t salt, bool fused = false) {
  az_mcts* m = az_mcts_create(game, n, slots, 1.25, use_gnn);
  if (!m) return fail("create");
  const int A = az_mcts_action_size(m), cells = n * n;
  std::vector<int8_t> boards((size_t)slots * cells);
  std::vector<int32_t> lslots(slots), fin(slots);
  std::vector<float> pi((size_t)slots * A), v(slots), gpi((size_t)slots * A), gv(slots);
  int started = 0, finished = 0, rounds = 0, held = 0;   // held: rows kept for feed_collect
  for (int s = 0; s < slots && started < episodes; ++s, ++started)
    if (az_mcts_episode_begin(m, s, 1000u + (uint32_t)started, sims, 3, 4)) return fail("begin");
  while (finished < episodes) {
    if (++rounds > 200000) return fail("no progress");
    const int k = held > 0
        ? az_mcts_feed_collect(m, held, pi.data(), v.data(), use_gnn ? gpi.data() : nullptr,
                               use_gnn ? gv.data() : nullptr, boards.data(), lslots.data(), slots,
                               threads)
        : az_mcts_collect(m, boards.data(), lslots.data(), slots, threads);
    held = 0;
    if (k < 0) return fail("collect");
    if (k > 0) {
      for (int i = 0; i < k; ++i) {
        fake_net(&boards[(size_t)i * cells], cells, A, salt, &pi[(size_t)i * A], &v[i]);
        fake_net(&boards[(size_t)i * cells], cells, A, salt ^ 0x5555, &gpi[(size_t)i * A], &gv[i]);
      }
      // an occasional failed batch: leaves degrade, an expand_tree root predict aborts
      const bool failed = (mix(salt + rounds) % 97) == 0;
      if (fused && !failed) {
        held = k;                        // fed by the next round's feed_collect
        goto harvest;
      }
      {
      const int rc = az_mcts_feed(m, k, pi.data(), v.data(), use_gnn ? gpi.data() : nullptr,
                                  use_gnn ? gv.data() : nullptr, failed ? 1 : 0);
      if (rc < 0) return fail("feed");
      if (rc > 0) {                      // aborted episodes: restart those slots fresh
        for (int s = 0; s < slots; ++s) {
          const int mv = az_mcts_episode_moves(m, s);
          if (mv < 0) return fail("moves");
        }
      }
      }
    }
  harvest:
    const int f = az_mcts_episode_finished(m, fin.data(), slots);
    if (f < 0) return fail("finished");
    if (fused && f > 0) {                // the batched export of all of them
      std::vector<int32_t> mvs(f);
      if (az_mcts_episodes_moves(m, fin.data(), f, mvs.data())) return fail("episodes_moves");
      size_t tot = 0;
      for (int i = 0; i < f; ++i) tot += (size_t)mvs[i];
      std::vector<int8_t> b(tot * cells), cur(tot), temp(tot), has(tot * A), tag(tot * A), vt(tot);
      std::vector<int32_t> act(tot), inn(tot * A), xn(tot * A);
      std::vector<double> p(tot * A), xq(tot * A), ip(tot * A), xp(tot * A), xv(tot), res(f);
      std::vector<float> sv(tot);
      std::vector<int> rt(f);
      if (az_mcts_episode_records(m, fin.data(), f, b.data(), cur.data(), temp.data(), act.data(),
                                  p.data(), inn.data(), has.data(), sv.data(), xn.data(), xq.data(),
                                  tag.data(), rt.data(), res.data(),
                                  use_gnn ? ip.data() : nullptr, use_gnn ? xp.data() : nullptr,
                                  use_gnn ? vt.data() : nullptr, use_gnn ? xv.data() : nullptr))
        return fail("episode_records");
    }
    for (int i = 0; i < f; ++i) {
      const int s = fin[i];
      const int mv = az_mcts_episode_moves(m, s);
      if (mv <= 0) return fail("moves of a finished episode");
      std::vector<int8_t> b((size_t)mv * cells), cur(mv), temp(mv), has((size_t)mv * A),
          tag((size_t)mv * A), vt(mv);
      std::vector<int32_t> act(mv), inn((size_t)mv * A), xn((size_t)mv * A);
      std::vector<double> p((size_t)mv * A), xq((size_t)mv * A), ip((size_t)mv * A),
          xp((size_t)mv * A), xv(mv);
      std::vector<float> sv(mv);
      int rt = 0;
      double res = 0;
      if (az_mcts_episode_record(m, s, b.data(), cur.data(), temp.data(), act.data(), p.data(),
                                 inn.data(), has.data(), sv.data(), xn.data(), xq.data(),
                                 tag.data(), &rt, &res))
        return fail("record");
      if (use_gnn && az_mcts_episode_targets(m, s, ip.data(), xp.data(), vt.data(), xv.data()))
        return fail("targets");
      ++finished;
      if (started < episodes) {
        if (az_mcts_episode_begin(m, s, 1000u + (uint32_t)started, sims, 3, 4))
          return fail("begin");
        ++started;
      }
    }
    if (k == 0 && f == 0) {
      // every remaining slot was aborted by a failed root predict: start them again
      for (int s = 0; s < slots && finished + 0 < episodes; ++s) {
        if (az_mcts_reset(m, s)) return fail("reset");
        if (started < episodes) {
          if (az_mcts_episode_begin(m, s, 7000u + (uint32_t)started, sims, 3, 4))
            return fail("begin");
          ++started;
        } else {
          ++finished;                    // an aborted episode that will not be replayed
        }
      }
    }
  }
  az_mcts_destroy(m);
  return 0;
}

// Search mode (NativeMCTS / ArenaPlayer): begin / collect / feed, root statistics, std cache.
int run_search(int game, int n, int use_gnn) {
  az_mcts* m = az_mcts_create(game, n, 2, 1.0, use_gnn);
  if (!m) return fail("create");
  const int A = az_mcts_action_size(m), cells = n * n;
  std::vector<int8_t> root(cells, 0), boards(2 * cells);
  std::vector<int32_t> sl(2), nsa(A), rem(2);
  std::vector<double> q(A);
  std::vector<int8_t> tag(A);
  std::vector<float> pi(2 * A), v(2), gpi(2 * A), gv(2);
  for (int move = 0; move < 6; ++move) {
    if (az_mcts_clear_predictions(m, 0)) return fail("clear");
    if (az_mcts_begin(m, 0, root.data(), 30)) return fail("begin");
    if (az_mcts_begin(m, 0, root.data(), 3) != AZM_ESTATE) return fail("double begin accepted");
    for (int it = 0; az_mcts_remaining(m, 0) > 0; ++it) {
      if (it > 10000) return fail("search stalls");
      const int k = az_mcts_collect(m, boards.data(), sl.data(), 2, 2);
      if (k < 0) return fail("collect");
      for (int i = 0; i < k; ++i) {
        fake_net(&boards[(size_t)i * cells], cells, A, 3, &pi[(size_t)i * A], &v[i]);
        fake_net(&boards[(size_t)i * cells], cells, A, 4, &gpi[(size_t)i * A], &gv[i]);
      }
      // speculative rows for the leaves' children (az_mcts_cache_put): later searches that
      // reach them expand inside collect
      for (int i = 0; i < k && it % 3 == 0; ++i) {
        std::vector<int8_t> kids((size_t)8 * cells);
        const int nk = az_game_children(game, n, &boards[(size_t)i * cells], 8, kids.data());
        if (nk < 0) return fail("children");
        std::vector<float> kp((size_t)nk * A + 1), kv(nk + 1), kg((size_t)nk * A + 1), kgv(nk + 1);
        for (int c = 0; c < nk; ++c) {
          fake_net(&kids[(size_t)c * cells], cells, A, 3, &kp[(size_t)c * A], &kv[c]);
          fake_net(&kids[(size_t)c * cells], cells, A, 4, &kg[(size_t)c * A], &kgv[c]);
        }
        if (az_mcts_cache_put(m, nk, kids.data(), kp.data(), kv.data(), kg.data(), kgv.data()))
          return fail("cache_put");
      }
      if (k && az_mcts_feed(m, k, pi.data(), v.data(), gpi.data(), gv.data(), it % 13 == 5) < 0)
        return fail("feed");
      if (az_mcts_remaining_all(m, rem.data())) return fail("remaining_all");
    }
    if (az_mcts_root_edges(m, 0, root.data(), nsa.data(), q.data(), tag.data()))
      return fail("root_edges");
    float sv = 0.f;
    if (az_mcts_get_std(m, 0, root.data(), &sv) < 0) return fail("get_std");
    if (az_mcts_set_std(m, 0, root.data(), 0.25f)) return fail("set_std");
    int best = -1;
    for (int a = 0; a < A; ++a)
      if (tag[a] != AZM_TAG_NONE && (best < 0 || nsa[a] > nsa[best])) best = a;
    if (best < 0) break;
    std::vector<int8_t> nxt(cells);
    int tagv = 0;
    double val = 0;
    if (az_game_next_canonical(game, n, root.data(), best, nxt.data())) return fail("next");
    root = nxt;
    if (az_game_ended(game, n, root.data(), &tagv, &val)) return fail("ended");
    if (val != 0.0) break;
  }
  int64_t st[4];
  if (az_mcts_tree_stats(m, 0, st)) return fail("tree_stats");
  int64_t cs[2];
  if (az_mcts_cache_stats(m, cs) || cs[0] <= 0) return fail("cache_stats");
  if (az_mcts_cache_clear(m) || az_mcts_cache_stats(m, cs) || cs[0] != 0) return fail("cache_clear");
  // error paths: bad slot, bad board, wrong feed count, feed without a collect
  std::vector<int8_t> bad(cells, 3);
  if (az_mcts_begin(m, 9, root.data(), 1) != AZM_EINVAL) return fail("bad slot accepted");
  if (az_mcts_begin(m, 1, bad.data(), 1) != AZM_EINVAL) return fail("bad board accepted");
  if (az_mcts_feed(m, 5, pi.data(), v.data(), gpi.data(), gv.data(), 0) != AZM_EINVAL)
    return fail("bad feed count accepted");
  az_mcts_destroy(m);
  return 0;
}

}  // namespace

int main() {
  if (az_mcts_create(0, 9, 1, 1.0, 0) != nullptr) return fail("n*n > 64 accepted");
  const int games[][2] = {{AZM_GAME_CONNECT4, 7}, {AZM_GAME_CONNECT4, 5},
                          {AZM_GAME_TICTACTOE, 3}, {AZM_GAME_TICTACTOE, 4}};
  for (const auto& g : games)
    for (int gnn = 0; gnn <= 1; ++gnn) {
      if (run_search(g[0], g[1], gnn)) return 1;
      for (int fused = 0; fused <= 1; ++fused)
        if (run_episodes(g[0], g[1], 5, gnn, 3, 9, g[0] == AZM_GAME_CONNECT4 ? 12 : 8,
                         (uint64_t)(g[0] * 131 + g[1] * 7 + gnn), fused != 0))
          return 1;
    }
  double a[37];
  for (int i = 0; i < 37; ++i) a[i] = i * 0.25;
  if (az_np_pairwise_sum(a, 37) != 166.5) return fail("pairwise sum");
  int64_t out[64];
  double p[5] = {0.1, 0.2, 0.3, 0.15, 0.25};
  if (az_rng_test(5, 2, 64, p, 5, out)) return fail("rng");
  printf("mcts_sanitize: ok\n");
  return 0;
}
