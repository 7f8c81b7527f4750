"""Multi-process (gloo, world_size 2, CPU) tests of the sharded self-play plumbing:
game-id sharding covers [0, n) exactly once and the record gather reassembles
rank-local games into one id-ordered set, identical to a single-rank run."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from uttt_amd.distributed import PLY_DTYPE, gather_records, pack_records, shard, unpack_records


def _fake_records(ids):
    recs = []
    for g in ids:
        rng = np.random.RandomState(g)
        n = 5 + g % 7
        st = np.zeros(n, PLY_DTYPE.fields["state"][0])
        st["own"][:, 0] = rng.randint(0, 2**27, size=n)
        st["active"] = -1
        recs.append({"game": g, "states": st, "policies": rng.rand(n, 81), "actions": rng.randint(0, 81, n),
                     "values": rng.randint(-1, 2, n)})
    return recs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_games, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = shard(n_games, rank, world)
    merged = gather_records(_fake_records(range(b, e)))
    if rank == 0:
        np.save(os.path.join(out_dir, "merged.npy"), pack_records(merged))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_partitions_ids():
    for n in (0, 1, 7, 500, 32768):
        for w in (1, 2, 3, 8):
            ranges = [shard(n, r, w) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(w - 1))
            sizes = [e - b for b, e in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_pack_roundtrip():
    recs = _fake_records([3, 1, 2])
    back = unpack_records(pack_records(recs))
    assert [r["game"] for r in back] == [1, 2, 3]
    for r in back:
        src = next(x for x in recs if x["game"] == r["game"])
        assert np.array_equal(r["policies"], src["policies"]) and np.array_equal(r["actions"], src["actions"])


def test_gloo_gather_two_ranks(tmp_path):
    n_games = 23
    mp.spawn(_worker, args=(2, _free_port(), n_games, str(tmp_path)), nprocs=2, join=True)
    merged = np.load(tmp_path / "merged.npy")
    single = pack_records(_fake_records(range(n_games)))
    assert np.array_equal(merged, single)
