"""One rank of tests/test_a0_gpu_multirank.py (started as a fresh process by
the test, RANK / WORLD_SIZE / MASTER_* in the environment, before anything in
it touches a GPU): classify this rank's contiguous shard through the C ABI
on device 0 with its own context, read every rule's hit count and the stats
back through the C ABI, sum them over ranks with a gloo all-reduce (the
per-CPU sum of xdp-filter status, xdp-filter/xdp-filter.c:93-103), and on
rank 0 write the sums for the test to compare with one oracle pass.
Usage: python gpu_rank_worker.py OUTDIR VARIANT QT_MIN_KEYS"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

import numpy as np  # noqa: E402


def main():
    outdir, variant, qmin = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    import xftools as X
    import xfgpu as G
    import xfshard as S
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(os.path.join(outdir, "batch.npz"))
    data, lens, stride = z["data"], z["lens"], int(z["stride"])
    rules = X.RuleSet()
    rules.v4_keys, rules.v4_vals = z["v4_keys"], z["v4_vals"]
    rules.ports = z["ports"]
    start, cnt = S.shard_range(len(lens), world, rank)
    mine = np.ascontiguousarray(data.reshape(-1, stride)[start:start + cnt]).reshape(-1)
    f = G.Filter(X.VARIANT_FEATURES[variant], devices=[0], ipv4_capacity=1 << 16,
                 qt_min_keys=qmin)
    f.load_rules(rules)
    v = f.run(mine, lens[start:start + cnt], stride=stride)
    path = f.last_path()
    r = rules.prepared()
    h4 = (f.values_of(G.MAP_IPV4, r.v4_keys) >> np.uint64(6)).astype(np.int64) - \
        (r.v4_vals >> np.uint64(6)).astype(np.int64)
    hp = (f.values_of(G.MAP_PORTS, np.arange(65536, dtype=np.uint32)) >> np.uint64(6)).astype(np.int64) - \
        (r.ports >> np.uint64(6)).astype(np.int64)
    st = f.stats().reshape(-1).astype(np.int64)
    f.close()
    flat = torch.from_numpy(np.concatenate([h4, hp, st]))
    dist.all_reduce(flat)                                  # SUM over ranks
    vs = [torch.zeros(S.shard_range(len(lens), world, q)[1], dtype=torch.uint8)
          for q in range(world)]
    dist.all_gather(vs, torch.from_numpy(v))
    paths = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(paths, torch.tensor([path], dtype=torch.int64))
    if rank == 0:
        np.savez(os.path.join(outdir, "sum.npz"), flat=flat.numpy(), verd=torch.cat(vs).numpy(),
                 paths=torch.cat(paths).numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
