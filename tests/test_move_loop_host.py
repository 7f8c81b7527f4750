"""CPU tests of SelfPlay's host bookkeeping around the C move loop (SelfPlay._steps_move_loop, round 6): a
scripted engine stands in for the GPU, so the order of the engine calls, the ring position, the counters and
the treatment of the last and of an empty move are pinned without a device. The GPU test
test_move_loop_in_c_equals_the_python_round_loop checks the same loop against the Python one and the oracle."""
import contextlib

import numpy as np
import pytest


class _Engine:
    """Moves scripted as (rounds enqueued, leaves, rounds with leaves); move_result reports the live slots of
    the next move from `live_after` (0 ends the games)."""

    def __init__(self, moves, live_after, live0=4):
        self.moves, self.live_after, self.live0 = list(moves), list(live_after), live0
        self.calls, self.ring = [], np.zeros((8, 4), np.int32)
        self.done = 0

    def count_ring(self):
        return self.ring

    def move_begin(self):
        self.calls.append("begin")
        return self.live0

    def rounds_hash_move(self, slot, policy, value, depth):
        self.calls.append(("rounds", slot, depth))
        return self.moves.pop(0)

    def move_end_async(self):
        self.calls.append("end_async")

    def move_begin_async(self):
        self.calls.append("begin_async")

    def move_result(self):
        self.calls.append("result")
        self.done += 1
        return self.done, self.live_after.pop(0)


class _Evaluator:
    rounds_per_call = 1

    def round_move(self, engine, slot, depth):
        return engine.rounds_hash_move(slot, None, None, depth)


class _Lane:
    def __init__(self, engine):
        self.engine, self.evaluator = engine, _Evaluator()
        self.count_ring, self.ring_pos, self.stream = None, 5, None
        self.leaves = self.rounds = self.finished = self.cur_live = 0


class _SP:
    evaluate_count = 30

    def __init__(self, lane):
        self.lanes, self.moves, self.sims = [lane], 0, 0

    @property
    def finished(self):
        return sum(ln.finished for ln in self.lanes)

    def _ctx(self, ln):
        return contextlib.nullcontext()


@pytest.fixture
def no_cuda_event(monkeypatch):
    import torch

    class _Ev:
        def record(self):
            pass

        def synchronize(self):
            pass

    monkeypatch.setattr(torch.cuda, "Event", _Ev)


def test_move_loop_counts_and_call_order(no_cuda_event):
    from uttt_amd.selfplay import SelfPlay
    e = _Engine([(9, 100, 7), (8, 90, 6), (10, 80, 7)], live_after=[4, 3, 3])
    ln = _Lane(e)
    sp = _SP(ln)
    seen = []
    total = SelfPlay._steps_move_loop(sp, ln, 3, 3, lambda f, _: seen.append(f))
    # three moves of 4, 4 and 3 live games (the second move's count is the first move's result)
    assert total == (4 + 4 + 3) * 30 and sp.sims == total and sp.moves == 3
    assert (ln.leaves, ln.rounds) == (270, 20)
    assert ln.ring_pos == 5 + 9 + 8 + 10  # every enqueued round consumed a ring slot
    assert e.calls == ["begin", ("rounds", 5, 3), "end_async", "begin_async", ("rounds", 6, 3), "result",
                       "end_async", "begin_async", ("rounds", 6, 3), "result", "end_async", "result"]
    assert seen == [1, 2, 3] and ln.finished == 3


def test_move_loop_stops_on_an_empty_move(no_cuda_event):
    from uttt_amd.selfplay import SelfPlay
    # the second move finds every game over (the first move's result: 0 live): its rounds ran, nothing counts
    e = _Engine([(9, 100, 7), (3, 0, 0)], live_after=[0])
    ln = _Lane(e)
    sp = _SP(ln)
    total = SelfPlay._steps_move_loop(sp, ln, None, 3, None)
    assert total == 4 * 30 and sp.moves == 1
    assert (ln.leaves, ln.rounds) == (100, 7)
    assert e.calls[-2:] == [("rounds", (5 + 9) % 8, 3), "result"]
    assert "end_async" in e.calls and e.calls.count("end_async") == 1


def test_move_loop_with_no_live_game_does_nothing(no_cuda_event):
    from uttt_amd.selfplay import SelfPlay
    e = _Engine([], live_after=[], live0=0)
    ln = _Lane(e)
    sp = _SP(ln)
    assert SelfPlay._steps_move_loop(sp, ln, 5, 3, None) == 0
    assert e.calls == ["begin"] and sp.moves == 0
