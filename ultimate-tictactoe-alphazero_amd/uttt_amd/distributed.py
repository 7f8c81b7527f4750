"""Multi-GPU self-play: one process per GPU, games sharded by global id.

Game g's result depends only on g (its RandomState(seed_base + g) stream and
the network), so sharding [0, n) into contiguous blocks per rank and gathering
the finished records at the end reproduces the single-GPU output exactly for
any world size. The data path has no collective; the only exchange is the
optional end-of-cycle gather of compact records to rank 0,
which rank 0 turns into the reference's .history list (train_network.py:21-24
reads only the newest file, so it must be one file).

Compact record per ply: packed state (32 B) + policy target (81 f64) +
action (i8) + value (i8) + game id (i64) = 690 B.
"""
import time

import numpy as np

from ._lib import STATE_DTYPE

PLY_DTYPE = np.dtype([("game", "<i8"), ("state", STATE_DTYPE), ("policy", "<f8", (81,)), ("action", "i1"),
                      ("value", "i1")])


def shard(n_games, rank, world):
    """Contiguous block [begin, end) of game ids for `rank` (sizes differ by at most one)."""
    base, extra = divmod(int(n_games), int(world))
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def pack_records(records):
    n = sum(len(r["actions"]) for r in records)
    out = np.zeros(n, PLY_DTYPE)
    i = 0
    for r in records:
        k = len(r["actions"])
        out["game"][i:i + k] = r["game"]
        out["state"][i:i + k] = r["states"]
        out["policy"][i:i + k] = r["policies"]
        out["action"][i:i + k] = r["actions"]
        out["value"][i:i + k] = r["values"]
        i += k
    return out


def unpack_records(plies):
    """Inverse of pack_records (plies of one game are contiguous, games sorted by id)."""
    plies = plies[np.argsort(plies["game"], kind="stable")]
    games, starts = np.unique(plies["game"], return_index=True)
    ends = list(starts[1:]) + [len(plies)]
    recs = []
    for g, a, b in zip(games.tolist(), starts.tolist(), ends):
        p = plies[a:b]
        recs.append({"game": g, "states": p["state"].copy(), "policies": p["policy"].copy(),
                     "actions": p["action"].astype(np.int64), "values": p["value"].astype(np.int64)})
    return recs


def gather_records(records, dst=0, group=None):
    """Gather every rank's finished games to `dst` (torch.distributed, any backend).
    Returns the merged records sorted by game id on dst, None elsewhere.

    Only dst receives: the ranks exchange their byte counts (one 8-byte all-gather), then
    every other rank sends its packed plies point-to-point to dst (RCCL send/recv over
    xGMI, or gloo on the CPU), which receives each into a buffer of exactly that size.
    No rank but dst allocates more than its own records."""
    import torch
    import torch.distributed as dist

    local = pack_records(records).view(np.uint8)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    n = torch.tensor([local.size], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    glob = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)  # noqa: E731
    if rank != dst:
        if local.size:
            dist.send(torch.from_numpy(local).to(dev), glob(dst), group=group)
        return None
    parts = [local.view(PLY_DTYPE)]
    for r in range(world):
        if r == rank or sizes[r] == 0:
            continue
        buf = torch.empty(sizes[r], dtype=torch.uint8, device=dev)
        dist.recv(buf, glob(r), group=group)
        parts.append(buf.cpu().numpy().view(PLY_DTYPE))
    return unpack_records(np.concatenate(parts) if parts else np.zeros(0, PLY_DTYPE))


def records_to_inputs(records):
    """Add the (9,9,3) input tensors (uttt_game.cpp:244-280) from the packed states, on the host rules
    (one batched call for all plies)."""
    import ctypes

    from . import _lib
    lib = _lib.load()
    if not records:
        return records
    st = np.ascontiguousarray(np.concatenate([r["states"] for r in records]))
    x = np.zeros((len(st), 243), np.float32)
    _lib.check(lib.uttt_states_input_hwc(st.ctypes.data_as(ctypes.POINTER(_lib.UtttState)), len(st),
                                         x.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    o = 0
    for r in records:
        k = len(r["states"])
        r["inputs"] = x[o:o + k].reshape(k, 9, 9, 3)
        o += k
    return records


def init_from_env():
    """(rank, world, local_rank) from torchrun's environment; initialises the default process
    group when WORLD_SIZE > 1 (RCCL on a GPU, gloo otherwise; UTTT_DIST_BACKEND overrides)."""
    import os

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world <= 1:
        return 0, 1, local
    if torch.cuda.is_available():
        local = local % torch.cuda.device_count()  # more ranks than GPUs: ranks share them
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        # RCCL refuses two ranks on one device: ranks sharing GPUs use gloo
        shared = torch.cuda.is_available() and world > torch.cuda.device_count()
        backend = os.environ.get("UTTT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() and not shared
                                                          else "gloo")
        dist.init_process_group(backend)
    return dist.get_rank(), dist.get_world_size(), local


def broadcast_int(value, src=0):
    """One Python int from `src` to every rank (the shared seed_base)."""
    import torch
    import torch.distributed as dist
    backend = dist.get_backend()
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([int(value) if value is not None else 0], dtype=torch.int64, device=dev)
    dist.broadcast(t, src)
    return int(t.item())


def self_play_sharded(model, n_games, slots, seed_base, evaluate_count=50, batch_size=8, temperature=1.0,
                      lanes=None, progress=None, evaluator_kind=None, timings=None):
    """Run this rank's contiguous shard of game ids [0, n_games) and gather every rank's records to
    rank 0 (records with inputs on rank 0, None elsewhere). Game g plays from RandomState(seed_base + g)
    whatever the world size, so the gathered records equal a single-GPU run."""
    import torch
    import torch.distributed as dist

    from .selfplay import SelfPlay, default_lanes
    rank, world = dist.get_rank(), dist.get_world_size()
    b, e = shard(n_games, rank, world)
    recs = []
    if e > b:
        n_slots = max(1, min(slots, e - b))
        n_lanes = default_lanes(n_slots) if lanes is None else lanes
        if n_slots % n_lanes:
            n_lanes = 1
        dev = torch.cuda.current_device() if torch.cuda.is_available() else None
        sp = SelfPlay(n_slots, evaluate_count, batch_size, temperature, device=dev, model=model, lanes=n_lanes,
                      evaluator_kind=evaluator_kind)
        t = sp.run(b, e, seed_base, progress)
        if timings is not None:
            timings["games_s"] = t
            timings["sims"] = sp.sims
        recs = sp.records(with_inputs=False)
    t0 = time.perf_counter()
    out = gather_records(recs)
    t1 = time.perf_counter()
    out = records_to_inputs(out) if out is not None else None
    if timings is not None:
        timings.update(gather_s=t1 - t0, inputs_s=time.perf_counter() - t1)
    return out
