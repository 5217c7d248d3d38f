// Host-only timing of the native engine (episode mode, Connect4 7x7, use_gnn, 100 sims) with a
// constant network: rows per second of collect + feed on ONE thread.  Build and profile:
//   g++ -O3 -std=c++17 -fopenmp -ffp-contract=off -pg tools/probes/mcts_bench.cpp \
//       alphazero-gnn_amd/csrc/az_mcts.cpp -o /tmp/mcts_bench && /tmp/mcts_bench 256 && gprof ...
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/az_mcts.h"

int main(int argc, char** argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 256;
  const int threads = argc > 2 ? atoi(argv[2]) : 1;
  const int n = 7, cells = 49;
  az_mcts* m = az_mcts_create(AZM_GAME_CONNECT4, n, S, 1.0, 1);
  const int A = az_mcts_action_size(m);
  for (int s = 0; s < S; ++s) az_mcts_episode_begin(m, s, 1000u + s, 100, 5, 15);
  std::vector<int8_t> boards((size_t)S * cells);
  std::vector<int32_t> slots(S), fin(S);
  std::vector<float> pi((size_t)S * A), v(S, 0.01f);
  for (int i = 0; i < S * A; ++i) pi[i] = (float)((i % A) + 1) / (A * (A + 1) / 2);
  long rows = 0;
  int finished = 0, rounds = 0;
  double tc = 0, tf = 0;
  while (finished < S && rounds < 100000) {
    auto t0 = std::chrono::steady_clock::now();
    const int k = az_mcts_collect(m, boards.data(), slots.data(), S, threads);
    auto t1 = std::chrono::steady_clock::now();
    if (k < 0) return 1;
    if (k > 0 && az_mcts_feed(m, k, pi.data(), v.data(), pi.data(), v.data(), 0) < 0) return 2;
    auto t2 = std::chrono::steady_clock::now();
    tc += std::chrono::duration<double>(t1 - t0).count();
    tf += std::chrono::duration<double>(t2 - t1).count();
    rows += k;
    finished += az_mcts_episode_finished(m, fin.data(), S);
    ++rounds;
  }
  printf("slots %d threads %d rounds %d rows %ld finished %d collect %.3f us/row feed %.3f us/row\n",
         S, threads, rounds, rows, finished, tc / rows * 1e6, tf / rows * 1e6);
  az_mcts_destroy(m);
  return 0;
}
