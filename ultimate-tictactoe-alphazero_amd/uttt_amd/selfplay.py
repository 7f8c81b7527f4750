"""Batched self-play and batched search on the engine.

The reference plays SP_GAME_COUNT games one after another, each move one
search whose flushes call the network at batch <= 8 (self_play_cpp.py:104-130,
pv_mcts_cpp.py:37-87). Here all games of a shard advance together: each round
every live tree contributes its one pending leaf to a single network batch.
"""
import math
import time

import numpy as np
import torch

from .engine import Engine, initial_states


def _bucket(n, cap, quantum=256):
    """Round a batch up so the network sees few distinct shapes (MIOpen tuning)."""
    if n <= 64:
        b = 1 << max(0, math.ceil(math.log2(max(n, 1))))
    else:
        b = ((n + quantum - 1) // quantum) * quantum
    return min(b, cap)


class HashEvaluator:
    """Device hash evaluator (bit-reproducible; the parity and kernel-bench evaluator)."""

    def __init__(self, engine):
        self.engine = engine
        dev = torch.device("cuda", engine.device)
        self.policy = torch.zeros((engine.max_trees, 81), dtype=torch.float32, device=dev)
        self.value = torch.zeros((engine.max_trees, 1), dtype=torch.float32, device=dev)

    def __call__(self, x, n):
        self.engine.eval_hash(x, n, self.policy, self.value)
        return self.policy[:n], self.value[:n]


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


class BatchedSearch:
    """pv_mcts_scores (uttt_mcts.cpp:84-196) for many root states at once."""

    def __init__(self, max_trees, max_sims=50, device=None, cache_log2=0):
        self.engine = Engine(max_trees, max_sims, device)
        if cache_log2:
            self.engine.set_cache(cache_log2, 0)
        dev = torch.device("cuda", self.engine.device)
        self.x = torch.zeros((max_trees, 3, 9, 9), dtype=torch.float32, device=dev)
        self.rounds = 0

    def run(self, roots, evaluator, evaluate_count=50, batch_size=8):
        e = self.engine
        e.use_stream()
        e.search_begin(roots, evaluate_count, batch_size)
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


class SelfPlay:
    """Concurrent self-play of games [begin, end) with `slots` trees in flight.

    Game g draws its moves from numpy's legacy MT19937 seeded seed_base + g, so
    its record equals self_play_cpp.play after np.random.seed(seed_base + g)
    (same model), independent of slot count, shard or GPU count."""

    def __init__(self, slots, evaluate_count=50, batch_size=8, temperature=1.0, device=None, evaluator=None,
                 model=None, cache_log2=None, cache_clear_every=32):
        self.engine = Engine(slots, evaluate_count, device)
        if cache_log2 is None:  # ~512 entries per slot: a 32-move window of one game's leaves
            cache_log2 = min(21, max(12, int(math.ceil(math.log2(max(slots, 1)))) + 9))
        if cache_log2:
            self.engine.set_cache(cache_log2, cache_clear_every)
        self.slots = slots
        self.evaluate_count = evaluate_count
        self.batch_size = batch_size
        self.temperature = temperature
        dev = torch.device("cuda", self.engine.device)
        self.x = torch.zeros((slots, 3, 9, 9), dtype=torch.float32, device=dev)
        if evaluator is None:
            evaluator = HashEvaluator(self.engine) if model is None else NetworkEvaluator(model, slots)
        self.evaluator = evaluator
        self.sims = 0
        self.rounds = 0
        self.moves = 0
        self.finished = 0

    def begin(self, game_begin, game_end, seed_base, arena_plies=None):
        self.engine.use_stream()
        self.engine.selfplay_begin(game_begin, game_end, seed_base, self.temperature, self.evaluate_count,
                                   self.batch_size, arena_plies)
        self.sims = self.rounds = self.moves = 0
        self.finished = 0

    def step(self):
        """One move for every live game. Returns the simulations it ran (0 = all games over)."""
        e = self.engine
        live = e.move_begin()
        if live == 0:
            return 0
        x = self.x if getattr(self.evaluator, "needs_input", True) else None
        while True:
            n = e.select(x)
            if n == 0:
                break
            p, v = self.evaluator(self.x, n)
            e.apply(p, v)
            self.rounds += 1
        self.finished = e.move_end()
        self.moves += 1
        done = live * self.evaluate_count
        self.sims += done
        return done

    def run(self, game_begin, game_end, seed_base, progress=None):
        self.begin(game_begin, game_end, seed_base)
        t0 = time.time()
        while self.step():
            if progress:
                progress(self.finished, game_end - game_begin)
        return time.time() - t0

    def records(self, with_inputs=True):
        """Finished games sorted by id: dict of per-game lists."""
        ids, off, ln = self.engine.games()
        pl = self.engine.plies(with_inputs)
        out = []
        for g, o, n in zip(ids.tolist(), off.tolist(), ln.tolist()):
            rec = {"game": g, "actions": pl["actions"][o:o + n].astype(np.int64),
                   "policies": pl["policies"][o:o + n], "values": pl["values"][o:o + n].astype(np.int64),
                   "states": pl["states"][o:o + n]}
            if with_inputs:
                rec["inputs"] = pl["inputs_hwc"][o:o + n].reshape(n, 9, 9, 3)
            out.append(rec)
        return out


def history_from_records(records):
    """The reference .history schema (self_play_cpp.py:59, :95-99): a flat list of
    [input (9,9,3) f32, policy (81,) f64, value int] over games in id order."""
    hist = []
    for r in records:
        for i in range(len(r["actions"])):
            hist.append([r["inputs"][i], r["policies"][i], int(r["values"][i])])
    return hist


__all__ = ["BatchedSearch", "SelfPlay", "HashEvaluator", "NetworkEvaluator", "history_from_records",
           "initial_states"]
