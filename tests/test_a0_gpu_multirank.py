"""Multi-rank readiness on the library itself: two fresh
rank processes (this file sorts first among the GPU tests, so the ranks are
started before the test process itself touches a GPU), each with its own context on device 0, classify their
contiguous shards of one batch through the C ABI; their per-rule hit counts
and stats -- read back through the C ABI, QT-order counts folded -- summed
over ranks with a gloo all-reduce must equal one oracle pass over the whole
batch, and the gathered verdicts the oracle's.  (RCCL refuses two ranks on
one device, so the device-side all-reduce, xfg_comm_allreduce, runs at one
rank here and across GPUs only in the driver's 8-GPU run.)  Contract: the
per-CPU sum at readout, xdp-filter/xdp-filter.c:93-103.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import xftools as X

pytestmark = pytest.mark.gpu
WORLD = 2
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("variant,qmin,path", [("xdpfilt_dny_all", 1, 5),
                                               ("xdpfilt_dny_all", 0xffffffff, 2),
                                               ("xdpfilt_alw_ip", 1, 5)])
def test_two_ranks_library_counters_sum_to_one_pass(tmp_path, variant, qmin, path):
    rng = np.random.default_rng(91)
    v4 = X.rand_keys(92, 20000, 4)
    vals = np.full(len(v4), 2, np.uint64) | (rng.integers(0, 9, len(v4)).astype(np.uint64) << 6)
    ports = (np.arange(16, dtype=np.uint16) * 1031 + 53).astype(np.uint16)
    rules = X.RuleSet()
    rules.v4_keys, rules.v4_vals = v4, vals
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    data, lens = X.gen_workload(93, 3, 1 << 18, 64, v4=v4, ports=ports)
    np.savez(tmp_path / "batch.npz", data=data, lens=lens, stride=64, v4_keys=v4,
             v4_vals=vals, ports=rules.ports)
    port = _free_port()
    procs = []
    for r in range(WORLD):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "gpu_rank_worker.py"),
                                       str(tmp_path), variant, str(qmin)], env=env))
    codes = [p.wait(timeout=240) for p in procs]
    assert codes == [0] * WORLD, codes
    got = np.load(tmp_path / "sum.npz")
    assert (got["paths"] == path).all(), got["paths"]
    ov, orules, ost = X.run_oracle(X.VARIANT_FEATURES[variant], data, lens, rules, stride=64,
                                   nthreads=8)
    r0 = rules.prepared()
    h4 = (orules.v4_vals >> np.uint64(6)).astype(np.int64) - (r0.v4_vals >> np.uint64(6)).astype(np.int64)
    hp = (orules.ports >> np.uint64(6)).astype(np.int64) - (r0.ports >> np.uint64(6)).astype(np.int64)
    want = np.concatenate([h4, hp, ost.reshape(-1).astype(np.int64)])
    np.testing.assert_array_equal(got["verd"], ov)
    np.testing.assert_array_equal(got["flat"], want)
    assert h4.sum() > 10000
