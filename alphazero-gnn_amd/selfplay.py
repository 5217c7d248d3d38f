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
plays exactly the episode the sequential reference plays after np.random.seed(seed(e)) GIVEN
THE SAME NETWORK OUTPUTS PER BOARD, independent of G and of how episodes are spread over ranks
(tests/test_selfplay.py, with recorded outputs).  On the GPU a row's outputs depend on the
batch it rides in (the GEMM's split-K factor and tile are chosen by B): they equal the batch-1
call within 1e-5 (tests/test_gpu_kernels.py) but not bit for bit, as the reference's own
batch-1 vs batch-B CPU GEMMs are not.  A UCB near-tie can therefore resolve
differently for different G or rank counts; tests/test_gpu_selfplay.py measures the action
agreement and locates the first divergence.

Network failures follow the reference (uniform priors, value 0 per leaf, MCTS.py:195-200) and
are counted in nn_fallback; an expand_tree root predict that fails propagates (MCTS.py:108-113).
"""
import os

import numpy as np

import hostcpu
import nn_fallback
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
            # (each waiting leaf is degraded -- and counted -- in MCTS._evaluate_leaf_g)
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


class _Immediate:
    """A prediction computed synchronously (network without *_async entry points)."""

    def __init__(self, out=None, err=None):
        self.out, self.err = out, err

    def result(self):
        if self.err is not None:
            raise self.err
        return self.out


def _launch(nnet, boards, want_gnn, stream=None):
    fn = getattr(nnet, "predict_both_async" if want_gnn else "predict_batch_async", None)
    try:
        if fn is not None:
            return fn(boards) if stream is None else fn(boards, stream=stream)
        return _Immediate(_net_call(nnet, boards, want_gnn))
    except Exception as ex:
        return _Immediate(err=ex)


class _Lane:
    """One native engine and the episodes running in its slots."""

    def __init__(self, game, nnet, args, G, cpuct, use_gnn, threads, queue, seeds, results):
        from mcts_native import Engine
        self.game, self.nnet, self.args = game, nnet, args
        self.use_gnn, self.threads = use_gnn, threads
        self.eng = Engine(game, G, cpuct, use_gnn)
        self.queue, self.seeds, self.results = queue, seeds, results
        self.free = list(range(G))[::-1]
        self.gens = {}            # slot -> [episode, generator]
        self.searching = set()    # slots waiting for their engine searches
        self.predicting = {}      # slot -> board waiting for a standard prediction
        self.k, self.pred = 0, []
        self.rounds = self.rows = 0

    def _handle(self, slot, req):
        if req[0] == "search":
            self.eng.begin(slot, req[1], req[2])
            self.searching.add(slot)
        else:
            self.predicting[slot] = req[1]

    def _resume(self, slot, value=None, exc=None):
        e, gen = self.gens[slot]
        try:
            req = gen.throw(exc) if exc is not None else gen.send(value)
        except StopIteration as stop:
            self.results[e] = stop.value
            del self.gens[slot]
            self.free.append(slot)
            return
        self._handle(slot, req)

    def start(self):
        from mcts_native import NativeMCTS
        while self.queue and self.free:
            slot = self.free.pop()
            e = self.queue.pop()
            self.eng.reset(slot)
            rng = np.random.RandomState(self.seeds[e])
            gen = episode_g(self.game, self.args, NativeMCTS(self.eng, slot, self.game, self.args,
                                                             rng), rng)
            self.gens[slot] = [e, gen]
            try:
                req = next(gen)
            except StopIteration as stop:
                self.results[e] = stop.value
                del self.gens[slot]
                self.free.append(slot)
                continue
            self._handle(slot, req)

    def gather(self):
        """Advance the searches to their next leaves -> boards to evaluate (or None)."""
        self.k = self.eng.collect(self.threads)
        self.pred = list(self.predicting.items())
        self.predicting.clear()
        if not self.k and not self.pred:
            return None
        boards = self.eng.leaf_boards[:self.k]
        if self.pred:
            boards = np.concatenate([boards, np.stack([np.asarray(b, np.int8)
                                                       for _, b in self.pred])])
        self.rounds += 1
        self.rows += len(boards)
        return boards

    def deliver(self, pending):
        """Feed a finished prediction (or none), resume every slot that can move on."""
        if pending is not None:
            try:
                pi, v, gpi, gv = pending.result()
                err = None
            except Exception as ex:   # the reference's per-leaf degradation (MCTS.py:195-200)
                err = ex
            k = self.k
            if k:
                if err is None:
                    self.eng.feed(k, pi, v, gpi, gv)
                else:    # the engine first (so it is left consistent), then the count
                    self.eng.feed(k, failed=True)
                    nn_fallback.record("selfplay.native", err, k)
            for i, (slot, _) in enumerate(self.pred):
                if err is None:
                    self._resume(slot, (pi[k + i], v[k + i]))
                else:
                    self._resume(slot, exc=err)     # unguarded in the reference (MCTS.py:108-113)
        rem = self.eng.remaining_all()
        for s in [s for s in sorted(self.searching) if rem[s] == 0]:
            self.searching.discard(s)
            self._resume(s)
        self.start()

    def live(self):
        return bool(self.gens)


def play_episodes_native(game, nnet, args, episodes, seeds, parallel_games=256, threads=None,
                         stats=None, lanes=2):
    """play_episodes with the searches in the native engine (mcts_native.py, libaz_mcts.so).

    The games are split over `lanes` engines that take turns: while one lane's leaf batch is
    on the GPU (predict_*_async: pinned copies + kernels + an event), the host advances the
    other lane's searches to their next leaves (engine threads) and resumes its finished
    moves.  Every round of a lane is: collect its leaves (+ pending root predictions) -> ONE
    batched network launch -> feed -> resume.  Same per-episode results as play_episodes for
    any lane count or slot count (each game owns its RandomState and tree)."""
    import time
    threads = int(threads or hostcpu.threads_per_rank())
    use_gnn = bool(getattr(args, "use_gnn", False) if not isinstance(args, dict)
                   else args.get("use_gnn", False))
    cpuct = args["cpuct"] if isinstance(args, dict) else args.cpuct
    episodes = list(episodes)
    G = max(1, min(int(parallel_games), len(episodes) or 1))
    lanes = max(1, min(int(lanes), G))
    queue = episodes[::-1]
    results = {}
    per = [G // lanes + (1 if i < G % lanes else 0) for i in range(lanes)]
    L = [_Lane(game, nnet, args, n, cpuct, use_gnn, threads, queue, seeds, results) for n in per]
    for lane in L:
        lane.start()
    inflight = [None] * lanes
    t0 = time.perf_counter()
    t_wait = 0.0
    idle = 0
    i = 0
    while any(lane.live() for lane in L) or any(x is not None for x in inflight):
        lane = L[i]
        if inflight[i] is not None:
            tw = time.perf_counter()
            p, inflight[i] = inflight[i], None
            if hasattr(p, "event"):
                p.event.synchronize()
            t_wait += time.perf_counter() - tw
            lane.deliver(p)
            idle = 0
        if lane.live():
            boards = lane.gather()
            if boards is not None:
                inflight[i] = _launch(nnet, boards, use_gnn)
                idle = 0
            else:
                lane.deliver(None)          # searches that finished without a leaf
                idle += 1
                if idle > 4 * lanes + 4 and not any(x is not None for x in inflight):
                    if all(not ln.live() for ln in L):
                        break
                    raise RuntimeError("native self-play made no progress (engine/driver bug)")
        i = (i + 1) % lanes
    if stats is not None:
        stats.update(rounds=sum(ln.rounds for ln in L), rows=sum(ln.rows for ln in L),
                     net_s=t_wait, host_s=time.perf_counter() - t0 - t_wait, lanes=lanes)
    return results


# live games per engine thread below which a lane's round uses fewer threads (0, the default:
# always all; AZ_SP_TAIL_SLOTS_PER_THREAD=16 measured equal in tools/gpu_sp_tail.sh's A/B)
_TAIL_SLOTS_PER_THREAD = int(os.environ.get("AZ_SP_TAIL_SLOTS_PER_THREAD", "0"))


class _EpisodeLane:
    """One native engine running whole episodes in its slots (engine episode mode)."""

    def __init__(self, game, args, G, cpuct, use_gnn, threads, queue, seeds, results, sims,
                 expand_by, temp_threshold):
        from mcts_native import Engine
        self.game, self.args, self.threads = game, args, threads
        self.eng = Engine(game, G, cpuct, use_gnn)
        self.queue, self.seeds, self.results = queue, seeds, results
        self.sims, self.expand_by, self.temp_threshold = sims, expand_by, temp_threshold
        self.free = list(range(G))[::-1]
        self.running = {}          # slot -> episode
        self.k = 0
        self.rounds = self.rows = 0
        self.assemble_s = 0.0
        self.collect_s = 0.0       # main-thread time inside the engine's (feed_)collect calls
        self.assembler, self.pending = None, []
        self.fed = None            # rows of the last batch, fed by the next gather

    def start(self):
        while self.queue and self.free:
            slot = self.free.pop()
            e = self.queue.pop()
            self.eng.episode_begin(slot, self.seeds[e], self.sims, self.expand_by,
                                   self.temp_threshold)
            self.running[slot] = e

    def harvest(self):
        """Finished slots: their records are copied out now (the slot is reused right away);
        the examples are assembled on the assembler thread when there is one (the engine's
        calls release the GIL, so assembly overlaps the search and the GPU wait)."""
        import time
        from mcts_native import assemble_episode
        t = time.perf_counter()
        fin = self.eng.episodes_finished()
        if fin:
            recs = self.eng.episode_records(fin)
            for slot, rec in zip(fin, recs):
                e = self.running.pop(slot)
                if self.assembler is None:
                    self.results[e] = assemble_episode(self.game, self.args, rec)
                else:
                    self.pending.append((e, self.assembler.submit(assemble_episode, self.game,
                                                                  self.args, rec)))
                self.free.append(slot)
        self.assemble_s += time.perf_counter() - t
        self.start()

    def finish(self):
        for e, f in self.pending:
            self.results[e] = f.result()
        self.pending = []

    def gather(self):
        import time
        t = time.perf_counter()
        # threads for this round's native pass: fewer once few games are left (each parallel
        # region wakes every sleeping worker; at the end of the run the work is a few descents)
        thr = self.threads
        if _TAIL_SLOTS_PER_THREAD > 0:
            thr = max(1, min(thr, len(self.running) // _TAIL_SLOTS_PER_THREAD))
        if self.fed is not None:        # last round's rows are fed inside this collect
            pi, v, gpi, gv = self.fed
            self.fed = None
            self.k = self.eng.feed_collect(self.k, pi, v, gpi, gv, thr)
        else:
            self.k = self.eng.collect(thr)
        self.collect_s += time.perf_counter() - t
        if not self.k:
            return None
        self.rounds += 1
        self.rows += self.k
        return self.eng.leaf_boards[:self.k]

    def deliver(self, pending):
        """A finished prediction: on success its rows are kept for the next gather
        (az_mcts_feed_collect: the feed and the next descents in one native pass; episodes only
        finish inside a collect, so harvesting first sees the same slots as feeding first)."""
        if pending is not None:
            try:
                pi, v, gpi, gv = pending.result()
            except Exception as err:  # the reference's per-leaf degradation (MCTS.py:195-200)
                aborted = self.eng.feed(self.k, failed=True)
                if aborted:
                    # expand_tree root predicts were in the batch: unguarded in the reference
                    # (MCTS.py:108-113), so the failure propagates out of those episodes -- after
                    # counting the batch's other leaves, which the same feed degraded (the feed
                    # returns how many of the k requests were aborted roots)
                    if self.k > aborted:
                        try:
                            nn_fallback.record("selfplay.engine", err, self.k - aborted)
                        except Exception:     # AZ_STRICT_NN: the original error wins
                            pass
                    raise err
                nn_fallback.record("selfplay.engine", err, self.k)
            else:                     # engine errors (shapes, state) propagate as themselves
                self.fed = (pi, v, gpi, gv)
        self.harvest()

    def live(self):
        return bool(self.running)


def play_episodes_engine(game, nnet, args, episodes, seeds, parallel_games=1024, threads=None,
                         stats=None, lanes=2, assembler_thread=True):
    """Whole self-play episodes in the native engine (episode mode, include/az_mcts.h): search,
    pi, move draws with each game's RandomState emulated draw for draw, expand_tree, rules --
    Python only batches the leaves for the network and assembles each finished game's
    examples.  Same results as play_episodes / Coach.executeEpisode per episode
    (tests/test_native_mcts.py)."""
    import time
    _ = _args_val(args, "numMCTSSims")
    threads = int(threads or hostcpu.threads_per_rank())
    use_gnn = bool(_args_val(args, "use_gnn", False))
    episodes = list(episodes)
    G = max(1, min(int(parallel_games), len(episodes) or 1))
    lanes = max(1, min(int(lanes), G))
    queue = episodes[::-1]
    results = {}
    per = [G // lanes + (1 if i < G % lanes else 0) for i in range(lanes)]
    L = [_EpisodeLane(game, args, n, _args_val(args, "cpuct"), use_gnn, threads, queue, seeds,
                      results, _args_val(args, "numMCTSSims"), _args_val(args, "expand_by", 5),
                      _args_val(args, "tempThreshold")) for n in per]
    pool = None
    if assembler_thread:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="az-assemble")
        for lane in L:
            lane.assembler = pool
    for lane in L:
        lane.start()
    streams = _lane_streams(nnet, use_gnn, lanes)
    inflight = [None] * lanes
    # diagnostics (tools/sp_pipeline_probe.py): stats["timeline"] = [] asks for one record per
    # lock-step round -- host times and the batch's GPU span from timing events on its stream
    tl_on = stats is not None and isinstance(stats.get("timeline"), list) and \
        streams[0] is not None
    if tl_on:
        import torch
        ref_ev = torch.cuda.Event(enable_timing=True)
        ref_ev.record()
        gpu_ev = []
    # The assembler thread runs Python while games finish; with the interpreter's default 5 ms
    # switch interval the lane loop's next launch waited for the GIL behind it (~1 ms per round
    # in the phase where most games end: tools/sp_pipeline_probe.py's timeline).  A short
    # interval hands the GIL back within ~0.2 ms.  AZ_SP_SWITCH_INTERVAL (seconds; 0 keeps the
    # interpreter's own) for A/B runs.
    import os
    import sys
    sw_old = sys.getswitchinterval()
    sw = float(os.environ.get("AZ_SP_SWITCH_INTERVAL", "0.0002"))
    if sw > 0:
        sys.setswitchinterval(sw)
    # the cyclic collector paused for the loop: finished games allocate example lists by the
    # thousand, and a full collection in the middle of a round stalled the next launch
    # (AZ_SP_GC=1 keeps it running, for A/B runs); reference cycles are collected after the loop.
    # The switch interval and the collector are process-wide: the lane loop owns them while it
    # runs, so one play_episodes_engine call at a time per process (the Coach and the bench
    # call it from one thread).
    import gc
    gc_was = gc.isenabled()
    if os.environ.get("AZ_SP_GC") != "1":
        gc.disable()
    t0 = time.perf_counter()
    t_wait = t_launch = 0.0
    idle = 0
    i = 0
    try:
        while any(lane.live() for lane in L) or any(x is not None for x in inflight):
            lane = L[i]
            rec = {"lane": i, "t_start": time.perf_counter() - t0} if tl_on else None
            if inflight[i] is not None:
                tw = time.perf_counter()
                p, inflight[i] = inflight[i], None
                if hasattr(p, "event"):
                    p.event.synchronize()
                t_wait += time.perf_counter() - tw
                if tl_on:
                    rec["wait"] = time.perf_counter() - tw
                lane.deliver(p)
                idle = 0
            if lane.live():
                boards = lane.gather()
                if boards is not None:
                    tl = time.perf_counter()
                    if tl_on:
                        e0, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(2))
                        e0.record(streams[i])
                    inflight[i] = _launch(nnet, boards, use_gnn, streams[i])
                    if tl_on:
                        e1.record(streams[i])
                        gpu_ev.append((len(stats["timeline"]), e0, e1))
                        rec.update(n=len(boards), t_launch=tl - t0,
                                   launch=time.perf_counter() - tl)
                    t_launch += time.perf_counter() - tl
                    idle = 0
                else:
                    lane.deliver(None)
                    idle += 1
                    if idle > 4 * lanes + 4 and not any(x is not None for x in inflight) and \
                            any(ln.live() for ln in L):
                        raise RuntimeError("native self-play made no progress (engine/driver bug)")
            if tl_on:
                stats["timeline"].append(rec)
            i = (i + 1) % lanes
        tf = time.perf_counter()
        for lane in L:
            lane.finish()
        drain_s = time.perf_counter() - tf
    finally:
        if pool is not None:
            pool.shutdown(wait=True)
        sys.setswitchinterval(sw_old)
        if gc_was and not gc.isenabled():
            gc.enable()
            gc.collect()      # the reference cycles the paused collector left behind
    if tl_on:
        torch.cuda.synchronize()
        for k, e0, e1 in gpu_ev:     # GPU span of each batch, ms from the reference event
            stats["timeline"][k].update(gpu_start=ref_ev.elapsed_time(e0) * 1e-3,
                                        gpu_end=ref_ev.elapsed_time(e1) * 1e-3)
    if stats is not None:
        stats["assemble_drain_s"] = drain_s
        stats.update(rounds=sum(ln.rounds for ln in L), rows=sum(ln.rows for ln in L),
                     net_s=t_wait, host_s=time.perf_counter() - t0 - t_wait, lanes=lanes,
                     assemble_s=sum(ln.assemble_s for ln in L),
                     collect_s=sum(ln.collect_s for ln in L), launch_s=t_launch)
    return results


def _lane_streams(nnet, use_gnn, lanes):
    """One HIP stream per lane for nets whose batched predict takes one (wrappers.py: each
    stream has its own device scratch), so a lane's batch can start while the other lane's is
    still on the GPU; every stream first waits for the work already queued on the current
    stream (parameter updates).  [None] * lanes otherwise (everything on the current stream)."""
    import inspect
    import os
    fn = getattr(nnet, "predict_both_async" if use_gnn else "predict_batch_async", None)
    if lanes < 2 or fn is None or "stream" not in inspect.signature(fn).parameters or \
            os.environ.get("AZ_SP_ONE_STREAM") == "1":
        return [None] * lanes
    import torch
    if not torch.cuda.is_available():
        return [None] * lanes
    cur = torch.cuda.current_stream()
    held = nnet.__dict__.setdefault("_lane_streams", [])   # reused: each owns device scratch
    while len(held) < lanes:
        held.append(torch.cuda.Stream())
    out = held[:lanes]
    for st in out:
        st.wait_stream(cur)
    return out


def _args_val(args, name, default=None):
    if isinstance(args, dict):
        return args.get(name, default)
    return getattr(args, name, default)
