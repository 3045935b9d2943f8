"""Gallery sharding + top-k exchange (opencv_facerecognizer_amd/parallel.py), world_size 2 on gloo (CPU).

The device merge kernel (ofr_topk_merge) is covered by tests/test_gpu_parity.py; here the
exchanged per-rank lists are merged by the oracle's stable ordering and must reproduce the
single-process global top-k exactly (indices and distances).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import facerec_oracle as O
from opencv_facerecognizer_amd.parallel import exchange_topk, shard_range, world


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    r = np.random.Generator(np.random.PCG64(7))
    G = r.normal(0, 1, (1001, 24))
    G[500] = G[17]                        # a tie across the shard boundary
    Q = r.normal(0, 1, (33, 24))
    Q[3] = G[17]
    return Q, G


def _worker(rank, ws, port, k, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        Q, G = _data()
        n0, n1 = shard_range(len(G), rank, ws)
        d, i = O.nn_search_vectorized("EuclideanDistance", Q, G[n0:n1], k)
        gd, gi = exchange_topk(torch.from_numpy(d), torch.from_numpy(i + n0))
        assert world() == (rank, ws)
        if rank == 0:
            out.put((gd.numpy(), gi.numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_disjointly():
    for N in (0, 1, 7, 1000, 1000001):
        for ws in (1, 2, 3, 8):
            rs = [shard_range(N, r, ws) for r in range(ws)]
            assert rs[0][0] == 0 and rs[-1][1] == N
            assert all(rs[j][1] == rs[j + 1][0] for j in range(ws - 1))


@pytest.mark.parametrize("k", [1, 4])
def test_two_rank_exchange_reproduces_global_topk(k):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, k, q)) for r in range(2)]
    for p in procs:
        p.start()
    gd, gi = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    Q, G = _data()
    ref_d, ref_i = O.nn_search_vectorized("EuclideanDistance", Q, G, k)
    assert gd.shape == (len(Q), 2 * k)
    for b in range(len(Q)):
        o = np.lexsort((gi[b], gd[b]))[:k]          # merge by (distance, index)
        assert np.array_equal(gi[b][o], ref_i[b]), b
        assert np.array_equal(gd[b][o], ref_d[b]), b
