"""Lock-step batched self-play: the caller side of the hot path.

The reference plays one game at a time and calls `predict` / `predict_with_gnn` on ONE board per
new MCTS leaf (MCTS.py:169-174, Coach.py:95-100): every network call is a batch of 1 with its
own host<->device copies.  Here G games run concurrently.  Each game is the same search
generator the sequential path uses (MCTS.py `*_g`, Coach.episode_g), so a game's search is
unchanged; the driver only decides WHEN leaves are evaluated:

    round:  every live game runs its host-side descent until it needs a leaf evaluation
            -> the G leaf boards go to the GPU as ONE predict_both / predict_batch call
            -> each game gets its own row back and continues.

A game that ends hands its slot to the next pending episode (continuous batching), so the
batch stays full until the last games drain.

Determinism: game e draws from its own np.random.RandomState(seed(e)) for both the move
choice (Coach.py:62) and MCTS's temp-0 tie-break (MCTS.py:39-44).  A lock-step game therefore
plays exactly the episode the sequential reference plays after np.random.seed(seed(e)) given
the same network outputs, independent of G and of how episodes are spread over ranks
(tests/test_selfplay.py).  Network outputs for a row of a batch equal the batch-1 call within
1e-5 (tests/test_gpu_kernels.py); they are not bit-identical, as the reference's own batch-1
vs batch-B CPU GEMMs are not.
"""
import os

import numpy as np

from Coach import episode_g
from MCTS import MCTS


class BatchEvaluator:
    """Serves a list of leaf requests [(board, want_gnn)] with one batched network call.

    Uses nnet.predict_both (one trunk pass, standard + GNN outputs) or nnet.predict_batch when
    the network has them; a plugin network without batch entry points is served row by row
    with its batch-1 predict / predict_with_gnn, exactly like the sequential path."""

    def __init__(self, nnet):
        self.nnet = nnet
        self.calls = 0
        self.rows = 0

    def __call__(self, requests):
        n = len(requests)
        self.calls += 1
        self.rows += n
        want_gnn = any(w for _, w in requests)
        fn = getattr(self.nnet, "predict_both" if want_gnn else "predict_batch", None)
        if fn is None:
            return [self._single(r) for r in requests]
        boards = np.stack([np.asarray(b) for b, _ in requests])
        try:
            out = fn(boards)
        except Exception as e:  # the reference degrades per leaf; a batch fails as a whole
            return [(None, None, e)] * n
        if want_gnn:
            pi, v, gpi, gv = out
            return [((pi[i], v[i]), (gpi[i], gv[i]) if requests[i][1] else None, None)
                    for i in range(n)]
        pi, v = out
        return [((pi[i], v[i]), None, None) for i in range(n)]

    def _single(self, request):
        board, want_gnn = request
        std = gnn = err = None
        try:
            std = self.nnet.predict(board)
            if want_gnn:
                gnn = self.nnet.predict_with_gnn(board)
        except Exception as e:
            err = e
        return std, gnn, err


def episode_seeds(base, episodes):
    """Per-episode RandomState seeds: a pure function of (base, episode index)."""
    return {e: (int(base) + e) % (1 << 32) for e in episodes}


def play_episodes(game, nnet, args, episodes, seeds, parallel_games=64, evaluator=None,
                  stats=None):
    """Play `episodes` (iterable of episode indices) with up to `parallel_games` live games.

    seeds: {episode: RandomState seed}.  Returns {episode: (std_examples, gnn_examples)}, each
    exactly what Coach.executeEpisode returns for that episode."""
    evaluator = evaluator or BatchEvaluator(nnet)
    pending = list(episodes)[::-1]
    live = []              # [episode, generator, pending request]
    results = {}

    def start():
        while pending and len(live) < max(1, parallel_games):
            e = pending.pop()
            rng = np.random.RandomState(seeds[e])
            mcts = MCTS(game, nnet, args, rng=rng)
            gen = episode_g(game, args, mcts, rng)
            try:
                live.append([e, gen, next(gen)])
            except StopIteration as stop:   # a game with no network call at all
                results[e] = stop.value

    start()
    rounds = 0
    while live:
        rounds += 1
        answers = evaluator([slot[2] for slot in live])
        still = []
        for slot, ans in zip(live, answers):
            try:
                slot[2] = slot[1].send(ans)
                still.append(slot)
            except StopIteration as stop:
                results[slot[0]] = stop.value
        live[:] = still
        start()
    if stats is not None:
        stats.update(rounds=rounds, rows=evaluator.rows, calls=evaluator.calls)
    return results


def _net_call(nnet, boards, want_gnn):
    """One batched network call -> (pi, v, gpi, gv) float32 arrays (gpi/gv None w/o GNN).
    Falls back to per-board calls for a plugin network without batch entry points."""
    if want_gnn and hasattr(nnet, "predict_both"):
        return nnet.predict_both(boards)
    if not want_gnn and hasattr(nnet, "predict_batch"):
        pi, v = nnet.predict_batch(boards)
        return pi, v, None, None
    std = [nnet.predict(b) for b in boards]
    pi = np.stack([p for p, _ in std]).astype(np.float32)
    v = np.array([x for _, x in std], np.float32)
    if not want_gnn:
        return pi, v, None, None
    g = [nnet.predict_with_gnn(b) for b in boards]
    return pi, v, np.stack([p for p, _ in g]).astype(np.float32), \
        np.array([x for _, x in g], np.float32)


def play_episodes_native(game, nnet, args, episodes, seeds, parallel_games=256, threads=None,
                         stats=None):
    """play_episodes with the searches in the native engine (mcts_native.py, libaz_mcts.so).

    Every round: the engine advances all slots' searches to their next new leaf (host
    threads), the leaves plus any pending root predictions go to the network as ONE batch,
    the results are fed back, and slots whose searches finished resume their episode logic
    (Coach.episode_g over NativeMCTS).  Same per-episode results as play_episodes."""
    import time
    from mcts_native import Engine, NativeMCTS
    threads = int(threads or min(16, os.cpu_count() or 1))
    use_gnn = bool(getattr(args, "use_gnn", False) if not isinstance(args, dict)
                   else args.get("use_gnn", False))
    cpuct = args["cpuct"] if isinstance(args, dict) else args.cpuct
    episodes = list(episodes)
    G = max(1, min(int(parallel_games), len(episodes) or 1))
    eng = Engine(game, G, cpuct, use_gnn)
    pending = episodes[::-1]
    free = list(range(G))[::-1]
    gens = {}             # slot -> [episode, generator]
    searching = set()     # slots waiting for their engine searches
    predicting = {}       # slot -> board waiting for a standard prediction
    results = {}
    t_net = t_host = 0.0
    rounds = rows = 0

    def handle(slot, req):
        if req[0] == "search":
            eng.begin(slot, req[1], req[2])
            searching.add(slot)
        else:
            predicting[slot] = req[1]

    def resume(slot, value=None, exc=None):
        e, gen = gens[slot]
        try:
            req = gen.throw(exc) if exc is not None else gen.send(value)
        except StopIteration as stop:
            results[e] = stop.value
            del gens[slot]
            free.append(slot)
            return
        handle(slot, req)

    def start():
        while pending and free:
            slot = free.pop()
            e = pending.pop()
            eng.reset(slot)
            rng = np.random.RandomState(seeds[e])
            gen = episode_g(game, args, NativeMCTS(eng, slot, game, args, rng), rng)
            gens[slot] = [e, gen]
            try:
                req = next(gen)
            except StopIteration as stop:
                results[e] = stop.value
                del gens[slot]
                free.append(slot)
                continue
            handle(slot, req)

    start()
    while gens:
        t0 = time.perf_counter()
        k = eng.collect(threads)
        pred = list(predicting.items())
        t1 = time.perf_counter()
        t_host += t1 - t0
        if k or pred:
            boards = eng.leaf_boards[:k]
            if pred:
                boards = np.concatenate([boards, np.stack([np.asarray(b, np.int8)
                                                           for _, b in pred])])
            try:
                pi, v, gpi, gv = _net_call(nnet, boards, use_gnn)
                err = None
            except Exception as ex:  # the reference's per-leaf degradation (MCTS.py:195-200)
                err = ex
            t2 = time.perf_counter()
            t_net += t2 - t1
            rounds += 1
            rows += len(boards)
            if k:
                if err is None:
                    eng.feed(k, pi, v, gpi, gv)
                else:
                    eng.feed(k, failed=True)
            predicting.clear()
            for i, (slot, _) in enumerate(pred):
                if err is None:
                    resume(slot, (pi[k + i], v[k + i]))
                else:
                    resume(slot, exc=err)     # unguarded in the reference (MCTS.py:108-113)
        t3 = time.perf_counter()
        rem = eng.remaining_all()
        done = [s for s in sorted(searching) if rem[s] == 0]
        for s in done:
            searching.discard(s)
            resume(s)
        start()
        t_host += time.perf_counter() - t3
        if not (k or pred or done) and gens:
            raise RuntimeError("native self-play made no progress (engine/driver state bug)")
    if stats is not None:
        stats.update(rounds=rounds, rows=rows, net_s=t_net, host_s=t_host)
    return results
