"""bench.py plumbing on CPU: the --gpus N launcher (rank processes, gloo barrier,
max-over-ranks timing, rank 0's JSON line) and the strong-scaling shard split, in
--dry-run mode (no GPU, no decode); tensor checks of the device decode entry points."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*args):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_launcher_two_ranks_dry_run():
    d = _run_bench("--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run")
    assert d["n_gpus"] == 2 and d["dry_run"] and d["scaling"] == "weak"
    assert d["metric"].startswith("codewords/s + info-bits/s") and d["roofline"]["kernel"] == "sclls_kernel<8>"
    # value = frames of all ranks / max wall over ranks
    assert d["value"] == pytest.approx(2 * 65536 * 3 / (d["ms_per_step"] * 3e-3), rel=1e-6)


def test_launcher_strong_scaling_shards():
    d = _run_bench("--gpus", "2", "--steps", "2", "--warmup", "0", "--dry-run", "--mode", "scl32_strong")
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["global_frames"] == 1 << 20 and d["roofline"]["kernel"] == "sclls_kernel<32>"
    assert d["roofline"]["frames_per_launch"] == 1 << 19  # rank 0's shard
    assert d["value"] == pytest.approx((1 << 20) * 2 / (d["ms_per_step"] * 2e-3), rel=1e-6)


def test_launcher_propagates_rank_failure():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--mode", "no_such_mode"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0


def test_src_digest_stable_and_traffic_stamp_rejected(tmp_path):
    sys.path.insert(0, ROOT)
    import bench
    d1, d2 = bench.src_digest(), bench.src_digest()
    assert d1 == d2 and len(d1) == 16
    t, why = bench.stamped_traffic("no_such_mode", "sclls_kernel<8>", d1)
    assert t is None and why == "no measurement"


def test_device_decode_rejects_bad_tensors():
    torch = pytest.importorskip("torch")
    from antpolarcodes_amd._native import Plan
    from antpolarcodes_amd.construction import frozen_bits
    fr = frozen_bits(128, 64, 0.0)
    p = Plan(128, 8, fr, crc=8, device=-1)  # host-only: the checks run before any HIP call
    llr = torch.zeros((4, 128), dtype=torch.float32)
    info = torch.zeros((4, 8), dtype=torch.uint8)
    with pytest.raises(ValueError, match="llr"):  # a CPU tensor is not on the plan's device
        p.decode_device(llr, info)
    with pytest.raises(ValueError, match="dtype"):
        p.decode_device(llr.to(torch.int8), info)
    with pytest.raises(ValueError, match="shape"):
        p.decode_device(torch.zeros((4, 64)), info)
    with pytest.raises(ValueError, match="contiguous"):
        p.decode_device(torch.zeros((128, 4)).t(), info)
    assert p.kernel_name() == "sclls_kernel<8>"
    assert Plan(128, 1, fr, device=-1).kernel_name() == "scq_kernel<16>"
    assert Plan(128, 1, fr, device=-1, fixed=True).kernel_name() == "sccs_kernel"
    assert Plan(128, 32, fr, device=-1, fixed=True).kernel_name() == "scl_char_kernel<32>"
    np.testing.assert_equal(p.kb, 8)
