// Host-only timing driver for the native MCTS engine (csrc/az_mcts.cpp): E Connect4 7x7 GNN
// episodes (sims 100, expand_by 5, tempThreshold 15) in lock step with a hash "network", fused
// feed_collect, `threads` OpenMP threads.  Prints simulations/s.  Build (gprof: add -pg):
//   g++ -O3 -std=c++17 -fopenmp -ffp-contract=off tools/native/mcts_prof.cpp \
//       alphazero-gnn_amd/csrc/az_mcts.cpp -o /tmp/mcts_prof && /tmp/mcts_prof 512 1
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <vector>

#include "../../include/az_mcts.h"

static uint64_t mix(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  return h ^ (h >> 33);
}

static void fake_net(const int8_t* b, int cells, int A, uint64_t salt, float* pi, float* v) {
  uint64_t h = salt;
  for (int i = 0; i < cells; ++i) h = mix(h + (uint64_t)(b[i] + 2) * 0x9e3779b97f4a7c15ULL);
  float s = 0.f;
  for (int a = 0; a < A; ++a) {
    h = mix(h + a);
    pi[a] = (float)((h >> 11) % 1000 + 1);
    s += pi[a];
  }
  for (int a = 0; a < A; ++a) pi[a] /= s;
  *v = (float)((int)(h % 2001) - 1000) / 1000.f;
}

int main(int argc, char** argv) {
  const int E = argc > 1 ? atoi(argv[1]) : 512, threads = argc > 2 ? atoi(argv[2]) : 1;
  const int n = 7, cells = n * n;
  az_mcts* m = az_mcts_create(AZM_GAME_CONNECT4, n, E, 1.0, 1);
  const int A = az_mcts_action_size(m);
  std::vector<int8_t> boards((size_t)E * cells);
  std::vector<int32_t> sl(E), fin(E);
  std::vector<float> pi((size_t)E * A), v(E), gpi((size_t)E * A), gv(E);
  for (int s = 0; s < E; ++s) az_mcts_episode_begin(m, s, 1000u + s, 100, 5, 15);
  int finished = 0, held = 0;
  long rows = 0, rounds = 0;
  const auto t0 = std::chrono::steady_clock::now();
  double tc = 0.0, tn = 0.0, tf = 0.0;
  while (finished < E) {
    const auto c0 = std::chrono::steady_clock::now();
    const int k = held > 0 ? az_mcts_feed_collect(m, held, pi.data(), v.data(), gpi.data(),
                                                  gv.data(), boards.data(), sl.data(), E, threads)
                           : az_mcts_collect(m, boards.data(), sl.data(), E, threads);
    tc += std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
    if (k < 0) { fprintf(stderr, "collect: %s\n", az_mcts_last_error()); return 1; }
    // the stand-in network runs on all threads (timed apart: it is not engine work -- serial,
    // it was 2.1-2.5 s of every 2,048-episode run and looked like an engine serial part)
    const auto n0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int i = 0; i < k; ++i) {
      fake_net(&boards[(size_t)i * cells], cells, A, 7, &pi[(size_t)i * A], &v[i]);
      fake_net(&boards[(size_t)i * cells], cells, A, 9, &gpi[(size_t)i * A], &gv[i]);
    }
    tn += std::chrono::duration<double>(std::chrono::steady_clock::now() - n0).count();
    held = k;
    rows += k;
    ++rounds;
    const auto f0 = std::chrono::steady_clock::now();
    const int f = az_mcts_episode_finished(m, fin.data(), E);
    tf += std::chrono::duration<double>(std::chrono::steady_clock::now() - f0).count();
    if (f < 0) { fprintf(stderr, "finished: %s\n", az_mcts_last_error()); return 1; }
    finished += f;
    if (k == 0 && f == 0 && held == 0) break;
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("episodes %d threads %d rounds %ld rows %ld seconds %.3f (in collect %.3f, stand-in net "
         "%.3f, episode_finished %.3f) episodes/s %.1f; engine-only (collect) episodes/s %.1f\n",
         E, threads, rounds, rows, dt, tc, tn, tf, E / dt, E / tc);
  az_mcts_destroy(m);
  return 0;
}
