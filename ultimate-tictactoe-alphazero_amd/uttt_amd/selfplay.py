"""Batched self-play and batched search on the engine.

The reference plays SP_GAME_COUNT games one after another, each move one
search whose flushes call the network at batch <= 8 (self_play_cpp.py:104-130,
pv_mcts_cpp.py:37-87). Here all games of a shard advance together: each round
every live tree contributes its one pending leaf to a single network batch.
"""
import collections
import contextlib
import math
import os
import time

import numpy as np
import torch

from .engine import Engine, RoundCount, initial_states


def _bucket(n, cap, quantum=256):
    """Round a batch up so the network sees few distinct shapes (MIOpen tuning)."""
    if n <= 64:
        b = 1 << max(0, math.ceil(math.log2(max(n, 1))))
    else:
        b = ((n + quantum - 1) // quantum) * quantum
    return min(b, cap)


class HashEvaluator:
    """Device hash evaluator (bit-reproducible; the parity and kernel-bench evaluator). With a
    RoundCount for n (device-count rounds) it reads the pending leaves' states and the count on the
    device (Engine.eval_hash_dev), so SelfPlay pipelines its rounds as with the fused network."""

    device_count = True
    cheap = True  # SelfPlay keeps two rounds in flight: the host's reaction, not the kernels, set the pace

    def __call__(self, x, n):
        if isinstance(n, RoundCount):
            self.engine.eval_hash_dev(self.policy, self.value)
            return self.policy, self.value
        self.engine.eval_hash(x, n, self.policy, self.value)
        return self.policy[:n], self.value[:n]

    def __init__(self, engine):
        self.engine = engine
        dev = torch.device("cuda", engine.device)
        self.policy = torch.zeros((engine.max_trees, 81), dtype=torch.float32, device=dev)
        self.value = torch.zeros((engine.max_trees, 1), dtype=torch.float32, device=dev)
        # rounds per C call (UTTT_ROUND_BATCH, default 1): a call may enqueue up to 4 one-dispatch rounds whose
        # last tag alone is polled, but the rounds enqueued past a move's end then outnumber the host time
        # saved: tree-only 4096 x 50, interleaved (profiles/r6/sweeps/u6j): 1 round per call, 3 in flight
        # 558-567M sims/s; 2 x 3 509-511M; 2 x 4 471-472M; 4 x 2 508-509M; 1 x 4 548-551M
        self.rounds_per_call = max(1, min(4, int(os.environ.get("UTTT_ROUND_BATCH", "1"))))

    def round_async(self, engine, slot):
        """rounds_per_call whole rounds in one C call (Engine.rounds_hash_async: per round one k_round1 launch
        that applies the previous round's evaluation, descends, evaluates the new leaves and publishes the
        counts; the last round's apply is staged for the next call or the move's end). SelfPlay.steps then
        polls the last round's tag in the host count ring instead of an event."""
        if self.rounds_per_call == 1:
            return engine.round_hash_async(slot, self.policy, self.value)
        return engine.rounds_hash_async(slot, self.policy, self.value, self.rounds_per_call)

    def round_move(self, engine, slot, depth):
        """A move's whole round loop in one C call (Engine.rounds_hash_move): `depth` rounds in flight, the
        host spinning on their tags in C, until a round leaves no tree with simulations."""
        return engine.rounds_hash_move(slot, self.policy, self.value, depth)


class NetworkEvaluator:
    """DualNetwork (or any model with its call signature) on the engine's device."""

    def __init__(self, model, max_batch):
        self.model = model
        self.max_batch = max_batch

    @torch.no_grad()
    def __call__(self, x, n):
        nb = _bucket(n, self.max_batch)
        p, v = self.model(x[:nb])
        return p[:n].float(), v[:n].float()


def model_evaluator_factory(model, kind=None):
    """make(engine) -> evaluator for a model: the fused HIP evaluator for a DualNetwork (the
    drop-ins' default, nnfast.evaluator_kind), else the model called on the engine's NCHW batch."""
    from .nnfast import FusedNetworkEvaluator, evaluator_kind
    if evaluator_kind(model, kind) == "fused":
        return lambda eng: FusedNetworkEvaluator(model, eng)
    return lambda eng: NetworkEvaluator(model, eng.max_trees)


class BatchedSearch:
    """pv_mcts_scores (uttt_mcts.cpp:84-196) for many root states at once."""

    def __init__(self, max_trees, max_sims=50, device=None, cache_log2=0):
        self.engine = Engine(max_trees, max_sims, device)
        if cache_log2:
            self.engine.set_cache(cache_log2, 0)
        dev = torch.device("cuda", self.engine.device)
        self.x = torch.zeros((max_trees, 3, 9, 9), dtype=torch.float32, device=dev)
        self.rounds = 0

    def run(self, roots, evaluator, evaluate_count=50, batch_size=8, semantics="cpp"):
        e = self.engine
        e.use_stream()
        e.search_begin(roots, evaluate_count, batch_size, semantics)
        self.rounds = 0
        x = self.x if getattr(evaluator, "needs_input", True) else None
        while True:
            n = e.select(x)
            if n == 0:
                break
            p, v = evaluator(self.x, n)
            e.apply(p, v)
            self.rounds += 1

    def scores(self, temperature):
        return self.engine.scores(temperature)

    def visits(self):
        return self.engine.root_visits()


class _TagReady:
    """Readiness of a one-call round: its ring slot's word 3 holds the round's tag (stored by k_scan or k_round1
    after the counts, which are drained first), polled like an event."""
    __slots__ = ("buf", "tag")

    def __init__(self, buf, tag):
        self.buf, self.tag = buf, tag

    def query(self):
        return int(self.buf[3]) == self.tag


class _Lane:
    """One engine + its stream, input buffer and evaluator."""

    def __init__(self, slots, evaluate_count, device, cache_log2, cache_clear_every, own_stream):
        self.engine = Engine(slots, evaluate_count, device)
        if cache_log2:
            self.engine.set_cache(cache_log2, cache_clear_every)
        # lanes run on their engines' own streams: streams created later (e.g. from
        # torch's pool) can share one of the few hardware queues and serialize
        self.stream = self.engine.own_stream() if own_stream else None
        dev = torch.device("cuda", self.engine.device)
        self.x = torch.zeros((slots, 3, 9, 9), dtype=torch.float32, device=dev)
        self.evaluator = None
        self.rounds = 0
        self.finished = 0
        self.count_ring = None  # pinned counts of the rounds in flight (async rounds, Engine.count_copy)
        self.ring_pos = 0
        self.spec = True        # enqueue the next round's network before its count is known
        self._no_rows = None
        self.leaves = 0         # pending leaves of this lane's rounds (the rows its evaluator was asked for)

    def no_rows(self):
        """(policy, value) device buffers for an apply with no pending leaf (nothing is read)."""
        if self._no_rows is None:
            dev = torch.device("cuda", self.engine.device)
            self._no_rows = (torch.zeros((1, 81), dtype=torch.float32, device=dev),
                             torch.zeros((1,), dtype=torch.float32, device=dev))
        return self._no_rows

    def use_stream(self):
        self.engine.use_stream(self.stream)


class SelfPlay:
    """Concurrent self-play of games [begin, end) with `slots` trees in flight.

    Game g draws its moves from numpy's legacy MT19937 seeded seed_base + g, so
    its record equals self_play_cpp.play after np.random.seed(seed_base + g)
    (same model), independent of slot count, shard or GPU count.

    lanes > 1 splits the slots (and the game range) over that many engines, each
    on its own HIP stream with its own evaluator. A step round-robins the lanes:
    while the host waits for one lane's pending count, the other lanes' network
    evaluations run, and their convolution kernels fill each other's partial
    last waves on the GPU. Records are unchanged (each game depends only on its id)."""

    def __init__(self, slots, evaluate_count=50, batch_size=8, temperature=1.0, device=None, evaluator=None,
                 model=None, cache_log2=None, cache_clear_every=0, lanes=1, evaluator_kind=None):
        if lanes < 1 or slots % lanes:
            raise ValueError("slots must be a positive multiple of lanes")
        per = slots // lanes
        if cache_log2 is None:  # ~2048 entries per slot (2^23 = 3 GB of HBM for 4096 games)
            cache_log2 = min(23, max(12, int(math.ceil(math.log2(max(per, 1)))) + 11))
        self.lanes = []
        for i in range(lanes):
            self.lanes.append(_Lane(per, evaluate_count, device, cache_log2 if i == 0 else 0, cache_clear_every,
                                    lanes > 1))
            if i and cache_log2:  # one table for all lanes: games in different lanes share positions
                self.lanes[i].engine.share_cache(self.lanes[0].engine)
        self.engine = self.lanes[0].engine
        self.x = self.lanes[0].x
        self.slots = slots
        self.evaluate_count = evaluate_count
        self.batch_size = batch_size
        self.temperature = temperature
        if evaluator is None and model is not None:
            self.set_evaluator(model_evaluator_factory(model, evaluator_kind))
        elif evaluator is None:
            self.set_evaluator(HashEvaluator)
        else:
            self.evaluator = evaluator
        self.sims = 0
        self.moves = 0
        self.cache_clear_every = cache_clear_every  # periodic clears need the blocking move boundary
        # rounds without a per-round host sync when every lane's evaluator reads the count on
        # the device (FusedNetworkEvaluator); UTTT_ASYNC_ROUNDS=0 keeps the blocking loop
        self.async_rounds = os.environ.get("UTTT_ASYNC_ROUNDS", "1") != "0"

    # one evaluator object per lane (each owns its buffers); with one lane the
    # attribute form is kept for compatibility
    def set_evaluator(self, make):
        """make(engine) -> evaluator, called once per lane. A new evaluator may compute other
        values: the shared evaluation table is cleared (its owner is lane 0)."""
        for ln in self.lanes:
            ln.evaluator = make(ln.engine)
        self.lanes[0].engine.cache_clear()

    @property
    def evaluator(self):
        return self.lanes[0].evaluator

    @evaluator.setter
    def evaluator(self, ev):
        if len(self.lanes) > 1:
            raise ValueError("with lanes > 1 use set_evaluator(make) (one evaluator per lane)")
        self.lanes[0].evaluator = ev

    @property
    def rounds(self):
        return sum(ln.rounds for ln in self.lanes)

    @property
    def finished(self):
        return sum(ln.finished for ln in self.lanes)

    @property
    def leaves(self):
        """Pending leaves of all rounds the device-count loop (steps) read back."""
        return sum(ln.leaves for ln in self.lanes)

    def _ctx(self, ln):
        return torch.cuda.stream(ln.stream) if ln.stream is not None else contextlib.nullcontext()

    def begin(self, game_begin, game_end, seed_base, arena_plies=None):
        n = len(self.lanes)
        span = game_end - game_begin
        for i, ln in enumerate(self.lanes):
            gb = game_begin + span * i // n
            ge = game_begin + span * (i + 1) // n
            if ln.stream is None:
                ln.engine.use_stream()
            else:
                ln.use_stream()
            with self._ctx(ln):
                ln.engine.selfplay_begin(gb, ge, seed_base, self.temperature, self.evaluate_count, self.batch_size,
                                         arena_plies if arena_plies is None else -(-arena_plies // n))
            ln.rounds = ln.finished = 0
        self.sims = self.moves = 0

    def _device_count(self):
        return (self.async_rounds and not self.cache_clear_every and
                all(getattr(ln.evaluator, "device_count", False) for ln in self.lanes))

    def step(self):
        """One move for every live game. Returns the simulations it ran (0 = all games over)."""
        if self._device_count():
            return self.steps(1)
        live = []
        for ln in self.lanes:
            with self._ctx(ln):
                live.append(ln.engine.move_begin())
        active = [ln for ln, n in zip(self.lanes, live) if n > 0]
        if not active:
            return 0
        queue = collections.deque(active)
        while queue:
            ln = queue.popleft()
            e = ln.engine
            with self._ctx(ln):
                x = ln.x if getattr(ln.evaluator, "needs_input", True) else None
                n = e.select(x)  # waits for this lane's previous round only
                if n == 0:
                    continue
                p, v = ln.evaluator(ln.x, n)
                e.apply(p, v)
                ln.rounds += 1
            queue.append(ln)
        for ln in active:
            with self._ctx(ln):
                ln.finished = ln.engine.move_end()
        self.moves += 1
        done = sum(live) * self.evaluate_count
        self.sims += done
        return done

    def steps(self, k=None, progress=None):
        """k moves of every lane (None: until every lane's games are over); returns the
        simulations run. With device-count evaluators (FusedNetworkEvaluator) the lanes are
        pipelined. A round's select, network and apply are enqueued without a host sync (the
        pending count stays on the device, Engine.select_async), and the host reads each round's
        counts back - a pinned copy right after the select's scan - only to decide whether to
        enqueue the next round (some tree has simulations left after this one) or end the move,
        while the current round's network still runs; so each lane's stream always holds work
        and no round is enqueued that would find nothing. A lane's move end and its next move's
        roots are enqueued the same way (Engine.move_end_async / move_begin_async; the counters
        are read when they have landed), so no lane idles at a move boundary, neither for the
        host nor for the other lane. Per lane the select launches
        are the blocking loop's minus its final empty one, each game depends only on its id,
        and every lane plays exactly k moves:
        records and totals are those of k lockstep steps (UTTT_ASYNC_ROUNDS=0)."""
        if not self._device_count():
            total, i = 0, 0
            while k is None or i < k:
                d = self.step()
                if d == 0:
                    break
                total += d
                i += 1
                if progress:
                    progress(self.finished, None)
            return total
        depth = self._lookahead()
        if (len(self.lanes) == 1 and depth > 1 and os.environ.get("UTTT_MOVE_LOOP", "1") != "0"
                and getattr(self.lanes[0].evaluator, "round_move", None) is not None
                and getattr(self.lanes[0].evaluator, "rounds_per_call", 1) == 1):
            return self._steps_move_loop(self.lanes[0], k, depth, progress)
        spin = depth > 1 and os.environ.get("UTTT_POLL_SLEEP", "0") != "1"
        for ln in self.lanes:
            if ln.count_ring is None:
                ln.count_ring = ln.engine.count_ring()  # the scan writes each round's counts here
            r = getattr(ln.evaluator, "rounds_per_call", 1)
            if len(ln.count_ring) < (depth + 1) * r and not (r > 1 and len(ln.count_ring) >= depth * r):
                raise ValueError(f"round look-ahead {depth} x {r} rounds per call needs more count slots")

        def fill(ln, q):
            # rounds in flight per lane: one (the next is enqueued once this one's count is read), or,
            # with a cheap evaluator, `depth`: the host's reaction then hides under the GPU's work; a
            # round enqueued past the move's last finds every tree done and changes nothing
            while len(q) < depth:
                q.append(self._enqueue_round(ln, ln.spec if depth == 1 else True))
            return q

        state = {}
        for ln in self.lanes:
            with self._ctx(ln):
                live = ln.engine.move_begin()  # the first move of the call: blocking, gives the live count
            if live > 0:
                ln.cur_live = live
                ln.moves_left = k
                ln.result_pending = False
                state[id(ln)] = (ln, fill(ln, collections.deque()))
        total = moves = 0
        while state:
            # serve whichever lane's oldest round count has landed (polling: waiting on one lane in
            # turn would leave the other lane's stream empty once it runs ahead)
            ready = [key for key in state if state[key][1][0][1].query()]
            if not ready:
                # cheap rounds (the hash evaluator, ~30 us each): spin, since a 20-us sleep lasts 60-100 us on
                # Linux and the three rounds in flight drain meanwhile (UTTT_POLL_SLEEP=1 sleeps as before)
                if not spin:
                    time.sleep(2e-5)
                continue
            for key in ready:
                ln, q = state[key]
                rc, ev, spec, buf = q.popleft()
                if ln.result_pending:  # the previous move's end: its counters landed before this count
                    ln.finished, ln.cur_live = ln.engine.move_result()
                    ln.result_pending = False
                    if progress:
                        progress(self.finished, None)
                if isinstance(buf, list):  # several rounds per call: leaves summed, the last round's `left`
                    n, more = sum(int(b[0]) for b in buf), int(buf[-1][2])
                else:
                    n, more = int(buf[0]), int(buf[2])
                rc.n = n
                ln.leaves += n
                if n > 0:
                    ln.rounds += 1
                if not spec:  # the network was held back until the count was known
                    with self._ctx(ln):
                        if n > 0:
                            p, v = ln.evaluator(None, rc)
                            ln.engine.apply(p, v)
                        else:
                            ln.engine.apply(*ln.no_rows())
                ln.spec = n > 0  # a round with leaves predicts another
                if ln.cur_live == 0:  # every game of the lane is over: this move was empty
                    # the rounds queued behind this one found no live tree either: their counts are 0
                    # (left unread, a RoundCount raises when a caller later sizes a batch by it)
                    for rc_empty, *_ in q:
                        rc_empty.n = 0
                    q.clear()
                    del state[key]
                    continue
                if more > 0:  # some tree has simulations left once this round is applied
                    fill(ln, q)
                    continue
                # this round completes the move (the rounds already enqueued behind it are empty: no
                # tree has a simulation left, so their counts are 0): end it and begin the next, both on
                # the stream, without waiting
                for rc_empty, *_ in q:
                    rc_empty.n = 0
                q.clear()
                total += ln.cur_live * self.evaluate_count
                moves += 1
                ln.moves_left = None if ln.moves_left is None else ln.moves_left - 1
                with self._ctx(ln):
                    ln.engine.move_end_async()
                    ln.result_pending = True
                    if ln.moves_left == 0:
                        ev_end = torch.cuda.Event()
                        ev_end.record()
                        ln.end_event = ev_end
                        del state[key]
                        continue
                    ln.engine.move_begin_async()
                fill(ln, q)
        for ln in self.lanes:  # the last move's counters
            if getattr(ln, "result_pending", False):
                ln.end_event.synchronize()
                ln.finished, ln.cur_live = ln.engine.move_result()
                ln.result_pending = False
                if progress:
                    progress(self.finished, None)
        self.moves += moves / len(self.lanes)
        self.sims += total
        return total

    def _steps_move_loop(self, ln, k, depth, progress):
        """steps() for one lane whose evaluator runs a move's rounds in one C call (HashEvaluator.round_move,
        round 6: tree-only self-play was bound by the host's per-round Python; UTTT_MOVE_LOOP=0 keeps the
        Python round loop). Per move: the round loop in C (`depth` rounds in flight, spinning on their tags),
        then the move's end and the next move's roots enqueued without waiting; the previous move's counters
        are read once the next move's first count has landed (its end ran before it on the stream). Same
        rounds, records and totals as the Python loop."""
        e = ln.engine
        if ln.count_ring is None:
            ln.count_ring = e.count_ring()
        with self._ctx(ln):
            live = e.move_begin()  # the first move of the call: blocking, gives the live count
        if live <= 0:
            return 0
        ln.cur_live = live
        total = moves = 0
        pending = False  # a move's end enqueued whose counters were not read yet
        while k is None or moves < k:
            n_rounds, leaves, with_leaves = ln.evaluator.round_move(e, ln.ring_pos % len(ln.count_ring), depth)
            ln.ring_pos += n_rounds
            if pending:  # the previous move's end ran before this move's first round
                ln.finished, ln.cur_live = e.move_result()
                pending = False
                if progress:
                    progress(self.finished, None)
            if ln.cur_live == 0:  # every game of the lane is over: this move was empty
                break
            ln.leaves += leaves
            ln.rounds += with_leaves
            total += ln.cur_live * self.evaluate_count
            moves += 1
            e.move_end_async()
            pending = True
            if k is not None and moves == k:
                break
            e.move_begin_async()
        if pending:
            with self._ctx(ln):
                ev = torch.cuda.Event()
                ev.record()
            ev.synchronize()
            ln.finished, ln.cur_live = e.move_result()
            if progress:
                progress(self.finished, None)
        self.moves += moves
        self.sims += total
        return total

    def _lookahead(self):
        """Rounds in flight per lane: UTTT_ROUND_LOOKAHEAD, else 3 when every lane's evaluator is cheap
        (the device hash evaluator: a round's kernels take about as long as the host's reaction to its
        count, so with one round in flight the GPU idled between rounds; with the fused rounds three in
        flight beat two in 3 of 3 interleaved runs, 395M against 387M sims/s,
        profiles/r5/ab/tree_shape/), else 1 (a network round is milliseconds: the host keeps up, and an
        empty look-ahead round would cost its 32 conv launches)."""
        env = os.environ.get("UTTT_ROUND_LOOKAHEAD")
        if env:
            return max(1, int(env))
        if not all(getattr(ln.evaluator, "cheap", False) for ln in self.lanes):
            return 1
        # calls in flight: their rounds' ring slots must not be reused before the call is read (8 slots)
        r = max(getattr(ln.evaluator, "rounds_per_call", 1) for ln in self.lanes)
        return 3 if r == 1 else max(1, 8 // r)

    def _enqueue_round(self, ln, spec):
        """Select of one round on the lane's stream, its counts stored by the scan into a slot of the
        engine's host count ring (no copy operation), and - speculatively, when the lane's previous round had leaves (always,
        with look-ahead) - the network and apply, all without a host sync. Otherwise (a lane whose
        rounds are answered by the cache or by terminal positions: the network would run empty) the
        host enqueues the network once the count shows leaves."""
        rc = RoundCount()
        slot = ln.ring_pos % len(ln.count_ring)
        buf = ln.count_ring[slot]
        one_call = getattr(ln.evaluator, "round_async", None)
        if spec and one_call is not None:
            # whole rounds in one C call, on the engine's stream; readiness is the tag the last round stores
            # into its ring slot after the counts (no event, no torch stream context per round). With several
            # rounds per call, the counts of the call's slots are summed (the last one's `left` decides)
            r = getattr(ln.evaluator, "rounds_per_call", 1)
            ln.ring_pos += r
            slots = [ln.count_ring[(slot + i) % len(ln.count_ring)] for i in range(r)]
            last = slots[-1]
            return rc, _TagReady(last, one_call(ln.engine, slot)), spec, (slots if r > 1 else last)
        ln.ring_pos += 1
        with self._ctx(ln):
            # readiness: the tag the scan stores into the ring slot after the counts (round 5; a torch event
            # per round before)
            if os.environ.get("UTTT_ROUND_EVENTS") == "1":  # the round-4 form, kept for A/B
                ln.engine.select_async_to(slot)
                ready = torch.cuda.Event()
                ready.record()
            else:
                ready = _TagReady(buf, ln.engine.select_async_tag(slot))
            if spec:
                p, v = ln.evaluator(None, rc)
                ln.engine.apply(p, v)
        return rc, ready, spec, buf

    def run(self, game_begin, game_end, seed_base, progress=None):
        self.begin(game_begin, game_end, seed_base)
        t0 = time.time()
        self.steps(None, (lambda f, _: progress(f, game_end - game_begin)) if progress else None)
        return time.time() - t0

    def kernel_stats(self, name):
        out = {"ms": 0.0, "launches": 0, "bytes": 0}
        for ln in self.lanes:
            st = ln.engine.kernel_stats(name)
            for k in out:
                out[k] += st[k]
        return out

    def cache_stats(self):
        out = {"hits": 0, "misses": 0, "inserts": 0, "replacements": 0}
        for ln in self.lanes:
            st = ln.engine.cache_stats()
            for k in out:
                out[k] += st[k]
        return out

    def set_timing(self, on=True):
        for ln in self.lanes:
            ln.engine.set_timing(on)

    def reset_stats(self):
        for ln in self.lanes:
            ln.engine.reset_stats()

    def records(self, with_inputs=True):
        """Finished games sorted by id: dict of per-game lists."""
        out = []
        for ln in self.lanes:
            ids, off, ln_ = ln.engine.games()
            pl = ln.engine.plies(with_inputs)
            for g, o, n in zip(ids.tolist(), off.tolist(), ln_.tolist()):
                rec = {"game": g, "actions": pl["actions"][o:o + n].astype(np.int64),
                       "policies": pl["policies"][o:o + n], "values": pl["values"][o:o + n].astype(np.int64),
                       "states": pl["states"][o:o + n]}
                if with_inputs:
                    rec["inputs"] = pl["inputs_hwc"][o:o + n].reshape(n, 9, 9, 3)
                out.append(rec)
        out.sort(key=lambda r: r["game"])
        return out


def default_lanes(slots):
    """Lanes the drop-ins use: two engines on two streams once the per-lane batch stays large
    (Lanes), one below that."""
    return 2 if slots >= 1024 and slots % 2 == 0 else 1


def history_from_records(records):
    """The reference .history schema (self_play_cpp.py:59, :95-99): a flat list of
    [input (9,9,3) f32, policy (81,) f64, value int] over games in id order."""
    hist = []
    for r in records:
        for i in range(len(r["actions"])):
            hist.append([r["inputs"][i], r["policies"][i], int(r["values"][i])])
    return hist


__all__ = ["BatchedSearch", "SelfPlay", "HashEvaluator", "NetworkEvaluator", "history_from_records",
           "initial_states", "model_evaluator_factory", "default_lanes"]
