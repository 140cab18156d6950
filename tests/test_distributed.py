"""N>1 path on CPU: world_size-2 gloo processes shard frames and reduce host stats
exactly as bench.py does on the GPU node (no data-path collective)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from antpolarcodes_amd.distributed import reduce_stats, shard_bounds


def test_shard_bounds_cover_exactly_once():
    for total in (1, 7, 1 << 20, 1000003):
        for ws in (1, 2, 3, 8):
            seen = np.zeros(total, np.int8)
            for r in range(ws):
                lo, hi = shard_bounds(total, ws, r)
                seen[lo:hi] += 1
            assert (seen == 1).all()
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    from pyoracle import Oracle
    from antpolarcodes_amd import frames
    from antpolarcodes_amd.construction import frozen_bits
    N, K, total = 64, 32, 96
    fr = frozen_bits(N, K, 0.0)
    llr, info, _ = frames.awgn_frames(N, fr, total, 3.0, seed=5, crc=8)  # same global batch everywhere
    lo, hi = shard_bounds(total, ws, rank)
    # each rank decodes only its shard; the oracle stands in for the GPU on this CPU test
    dec, ok = Oracle().scl_decode(N, 4, fr, llr[lo:hi], crc=8)
    errs = int((~(dec == info[lo:hi]).all(axis=1)).sum())
    st = reduce_stats({"frames": (hi - lo, "sum"), "errors": (errs, "sum"), "t": (0.1 * (rank + 1), "max")})
    if rank == 0:
        full, _ = Oracle().scl_decode(N, 4, fr, llr, crc=8)
        q.put((st, int((~(full == info).all(axis=1)).sum())))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharded_decode():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    st, full_errs = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert st["frames"] == 96
    assert st["errors"] == full_errs
    assert abs(st["t"] - 0.2) < 1e-12
