"""World-size-2 gloo tests of the multi-GPU decomposition on CPU: each rank
classifies its contiguous shard with the CPU restatement (oracle/), hits and
stats are summed with an all-reduce, and the result must equal one pass over
the whole batch — the property the RCCL path (xfg_comm_allreduce) relies on.
"""
import os
import socket

import numpy as np
import pytest

import xftools as X
import xfshard as S

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, outdir, variant):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rules, pool = X.random_rules(5, n4=300, n6=80, ne=30, nports=40)
    data, lens = X.gen_fuzz(21, 40000, 160, rules, pool)
    start, cnt = S.shard_range(len(lens), world, rank)
    mine = np.ascontiguousarray(data.reshape(-1, 160)[start:start + cnt]).reshape(-1)
    v, after, st = X.run_oracle(X.VARIANT_FEATURES[variant], mine, lens[start:start + cnt],
                                rules, stride=160)
    r0 = rules.prepared()
    # per-rank hit deltas (the rules start with non-zero hits: subtract them)
    parts = []
    for fld in ("ports", "v4_vals", "v6_vals", "eth_vals"):
        h1, _ = S.split_hits(getattr(after, fld))
        h0, _ = S.split_hits(getattr(r0, fld))
        parts.append((h1 - h0).astype(np.int64))
    flat = torch.from_numpy(np.concatenate(parts + [st.reshape(-1).astype(np.int64)]))
    dist.all_reduce(flat)                              # SUM
    vs = [torch.zeros(S.shard_range(len(lens), world, r)[1], dtype=torch.uint8)
          for r in range(world)]
    dist.all_gather(vs, torch.from_numpy(v))
    if rank == 0:
        np.save(os.path.join(outdir, "sum.npy"), flat.numpy())
        np.save(os.path.join(outdir, "verd.npy"), torch.cat(vs).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_ip"])
def test_two_rank_shards_sum_to_one_pass(tmp_path, variant):
    import torch.multiprocessing as mp
    mp.spawn(_rank_main, args=(WORLD, _free_port(), str(tmp_path), variant), nprocs=WORLD,
             join=True)
    rules, pool = X.random_rules(5, n4=300, n6=80, ne=30, nports=40)
    data, lens = X.gen_fuzz(21, 40000, 160, rules, pool)
    v, after, st = X.run_oracle(X.VARIANT_FEATURES[variant], data, lens, rules, stride=160)
    r0 = rules.prepared()
    want = []
    for fld in ("ports", "v4_vals", "v6_vals", "eth_vals"):
        h1, _ = S.split_hits(getattr(after, fld))
        h0, _ = S.split_hits(getattr(r0, fld))
        want.append((h1 - h0).astype(np.int64))
    want = np.concatenate(want + [st.reshape(-1).astype(np.int64)])
    np.testing.assert_array_equal(np.load(tmp_path / "sum.npy"), want)
    np.testing.assert_array_equal(np.load(tmp_path / "verd.npy"), v)


def test_shard_ranges_cover_batch():
    for n in (0, 1, 7, 1000, 2 ** 24 + 3):
        for w in (1, 2, 3, 8):
            spans = [S.shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_reduced_values_keep_own_flags():
    a = np.array([(5 << 6) | 2, (0 << 6) | 1], np.uint64)
    b = np.array([(7 << 6) | 3, (4 << 6) | 1], np.uint64)
    ra, rb = S.reduced_values([a, b])
    assert ra.tolist() == [(12 << 6) | 2, (4 << 6) | 1]
    assert rb.tolist() == [(12 << 6) | 3, (4 << 6) | 1]
