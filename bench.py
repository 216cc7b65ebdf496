#!/usr/bin/env python3
"""bench.py — headline benchmark: Mpps classified (device-resident), 64B
frames, xdpfilt_dny_all, 1M IPv4 rules (BASELINE.json configs[2] = "C3").

One step = one xfg_classify() launch over the whole synthetic batch resident
in HBM (2^26 packets of 64 B, a 4 GiB batch, per GPU by default).  N GPUs = N processes, one
per GPU, each with its own shard (rank-seeded batch; rule tables replicated):
weak scaling, no data-path collective.  Counters are reduced over RCCL once,
after the timed region (reported separately as reduce_ms).

Prints ONE JSON line on rank 0 (contract in the task statement), including
  roofline:     algorithmic bytes per launch (sum over packets of
                min(len,128)+1) / average kernel duration from
                HIP events on the launch stream, vs the 8 TB/s HBM peak
  cpu_baseline: the CPU restatement of xdpfilt_dny_all (oracle/, "port")
                with the reference's cost model (one hash probe per
                CHECK_MAP, per-thread counters summed) on a bounded sample
                of the same workload (N=1, rank 0 only), on all the host
                cores this process may use and on one; the CPU model is
                named.  The reference's own in-kernel run (C1) is
                not measured: it needs a BPF-capable clang, libbpf, bpffs,
                veth/iproute2 and root, none of which this image has.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

METRIC = "Mpps classified (device-resident), 64B frames, xdpfilt_dny_all; 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0
REDUCE_TIMEOUT_S = 120.0   # the readout all-reduce (outside the timed region)


# the classify kernel each launch path runs (xfg_last_path)
KERNEL_OF_PATH = {
    0: "xfg_classify_kernel (general)",
    1: "xfg_pipeline_kernel (generic pipelined)",
    2: "xfg_pipe4_kernel (IPv4-key pipelined)",
    5: "xfg_pipeq_kernel (IPv4-key pipelined over the quotient index)",
    6: "xfg_pipee_kernel (Ethernet-key, the map as an LDS key table)",
}
# rocprofv3 --pmc summaries of the bench's own workload (tools/pmc.sh,
# tools/pmc_summary.py): per launch path, the file and the batch it was taken at
# (round 5: the QT kernel with pending logs and the mask-free rings; a pass of an
# older kernel would misstate this one's traffic)
PMC_OF_PATH = {5: ("profiles/r06_c3_pmc_2p26.json", 1 << 26)}


def committed_traffic(path, n, stream_bytes):
    """HBM bytes per launch from the committed PMC passes of this path's
    kernel at this batch, or None when no such file matches.  gfx950's
    FETCH_SIZE tallies a wide coalesced read at half its bytes and a random
    32/64-byte line at its bytes (profiles/archive/r02_fetch_size_calibration.json),
    so the frame + length stream's other half is added back, not the whole
    figure doubled; WRITE_SIZE as read."""
    ent = PMC_OF_PATH.get(path)
    if not ent or ent[1] != n or not os.path.exists(os.path.join(ROOT, ent[0])):
        return None, "null: no committed PMC pass of this kernel at this batch"
    d = json.load(open(os.path.join(ROOT, ent[0])))
    if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
        return None, f"null: {ent[0]} lacks FETCH_SIZE/WRITE_SIZE"
    t = int(d["FETCH_SIZE"] * 1024 + stream_bytes / 2 + d["WRITE_SIZE"] * 1024)
    return t, (f"{ent[0]} (separate rocprofv3 --pmc runs of the same kernel and workload): "
               "FETCH_SIZE + half the frame/length stream (tallied at half on gfx950) "
               "+ WRITE_SIZE, per launch")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log2-packets", type=int, default=26)
    ap.add_argument("--rules", type=int, default=1_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU-baseline duration (0 disables)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal on a one-GPU box: every rank uses device 0 (RCCL then "
                         "refuses the shared device, which the line reports as reduce_error)")
    ap.add_argument("--host-log2-packets", type=int, default=22,
                    help="sample for the PCIe-inclusive host-buffer rate (0 disables)")
    ap.add_argument("--rank-timeout", type=float, default=1800.0,
                    help="self-launch (--gpus N without a launcher): seconds before the "
                         "ranks count as stalled")
    # launcher tests (CPU only): a rank body that touches no GPU
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stub-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--stub-stall-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--stub-reduce-stall-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--reduce-timeout", type=float, default=REDUCE_TIMEOUT_S,
                    help="seconds before the readout all-reduce counts as stalled")
    return ap.parse_args()


def launch_ranks(args, argv):
    """`--gpus N` with no launcher around it (WORLD_SIZE unset): start N fresh
    rank processes of this script -- RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT set, never exec, and before anything in this
    process touches a GPU -- relay rank 0's line (the other ranks' stdout goes
    to stderr), and return non-zero if any rank fails or the ranks stall past
    --rank-timeout (each rank is then killed by its own process group)."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=None if r == 0 else 2,
                                      start_new_session=True))

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        for p in procs:
            p.wait()

    deadline = time.monotonic() + args.rank_timeout
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            print(f"bench: a rank failed (exit {bad[0]}); stopping the others", file=sys.stderr)
            kill_all()
            return bad[0] if bad[0] > 0 else 1
        if all(c == 0 for c in codes):
            return 0
        if time.monotonic() > deadline:
            print(f"bench: ranks stalled past {args.rank_timeout:.0f}s; killed", file=sys.stderr)
            kill_all()
            return 124
        time.sleep(0.1)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if args.stub:
        sys.exit(stub_rank(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = init_gloo() if world > 1 else None   # gloo: CPU barriers / max only
    import numpy as np
    import xftools as X
    import xfgpu as G

    f, bufs, n, stride, lens, alg_bytes, v4, ports, gen_s = setup(args, rank,
                                                                  0 if args.one_device else local)
    d_data, d_lens, d_verd = bufs

    def barrier():
        if dist is not None:
            dist.barrier()

    # ---- warmup
    if args.warmup:
        f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_verd.ptr, args.warmup, lens_u16=True)
    f.sync()
    # ---- timed region: K launches back-to-back on the library's stream,
    # HIP events recorded on that stream around them
    barrier()
    f.sync()
    t1 = time.perf_counter()
    kern_ms = f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_verd.ptr, args.steps,
                               lens_u16=True)
    f.sync()
    barrier()
    wall = time.perf_counter() - t1
    wall = max_over_ranks(dist, wall)

    # ---- sanity on the run's own outputs (cheap, not a parity claim)
    st = f.stats(dev=0)
    assert int(st[:, 0].sum()) == n * (args.steps + args.warmup), st

    # ---- RCCL counter reduce (once, after the timed region)
    # (outside the timed region; a failure or a stall here is reported in the
    # line and never keeps the line from being printed)
    reduce_ms, reduce_err, reduce_stuck = None, None, False
    if world > 1:
        uid = [G.Filter.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)

        def _reduce():
            f.comm_init(world, rank, uid[0])
            f.sync()
            tr = time.perf_counter()
            f.comm_allreduce()
            f.sync()
            return (time.perf_counter() - tr) * 1e3

        reduce_ms, reduce_err, reduce_stuck = watched_reduce(_reduce, args.reduce_timeout)

    # ---- achievable streaming-read peak on this device (same 1 GiB buffer)
    peak_meas_ms = f.stream_read_timed(d_data.ptr, n * stride, 5)
    peak_meas = n * stride / (peak_meas_ms * 1e-3) / 1e9

    # ---- PCIe-inclusive rate: the same workload handed over in host memory
    # (xfg_classify_host: pinned staging, H2D, classify, D2H of verdicts);
    # reported beside `value`, never as it
    host_path = None
    if rank == 0 and args.host_log2_packets > 0:
        hn = 1 << args.host_log2_packets
        hdata, hlens = X.gen_workload(7, 3, hn, stride, v4=v4, ports=ports, dst_permille=500,
                                      port_permille=250, bad_permille=10)
        f.classify_host(hdata, hlens, stride=stride)          # warm the staging buffers
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            f.classify_host(hdata, hlens, stride=stride)
        hs = (time.perf_counter() - t0) / reps
        # the same batch registered once (xfg_host_register, as a long-lived
        # capture ring or UMEM would be): the kernels read its mapped pages
        # in place (zero copy), no staging
        f.host_register(hdata)
        f.classify_host(hdata, hlens, stride=stride)
        t0 = time.perf_counter()
        for _ in range(reps):
            f.classify_host(hdata, hlens, stride=stride)
        hr = (time.perf_counter() - t0) / reps
        f.host_unregister(hdata)
        host_path = {"Mpps": round(hn / hs / 1e6, 1), "packets": hn, "ms": round(hs * 1e3, 3),
                     "GBps_h2d": round(hdata.nbytes / hs / 1e9, 1),
                     "registered_Mpps": round(hn / hr / 1e6, 1),
                     "registered_GBps_h2d": round(hdata.nbytes / hr / 1e9, 1),
                     "gather_threads": int(G.lib.xfg_host_threads()),
                     "note": "host-resident batch incl. H2D frames+lens and D2H verdicts "
                             "(xfg_classify_host: pinned staging copy by the device's pool; "
                             "registered: the kernels read the caller's mapped pages in place)"}
        del hdata

    # ---- CPU baseline (rank 0, N=1 only)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_seconds > 0:
        cpu = cpu_baseline(X, np, v4, ports, args.cpu_seconds)

    # ---- traffic: PMC bytes cannot be counted inside this timed process
    # (a rocprofv3 --pmc pass is its own run): the per-launch figures of the
    # same kernel on the same workload, committed under profiles/ (DESIGN.md
    # §6), corrected as MI355X_MICROARCH.md's HBM section prescribes
    path = f.last_path()
    kname = KERNEL_OF_PATH.get(path, f"path {path}")
    traffic, traffic_src = committed_traffic(path, n, n * stride + n * 2)

    total_pkts = n * args.steps * world
    value = total_pkts / wall / 1e6
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "Mpps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded xorshift64*, tools/xfsynth.c)",
        "config": {
            "workload": "C3: xdpfilt_dny_all, 1M IPv4 dst rules + 16 dst-port rules (tcp|udp), "
                        "64B frames at 64B stride (80% IPv4/UDP, 10% IPv4/TCP, 10% IPv6/UDP 62B, "
                        "1% malformed), 50% dst-IP hits, u16 lens, device-resident",
            "packets_per_gpu": n,
            "rules_ipv4": args.rules,
            "program": f.prog_name,
            "parallelism": f"shard{world}",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "alg_bytes_per_launch": alg_bytes,
            "kernel_ms": round(kern_ms, 4),
            "kernel": f"one classify pass: {kname} + xfg_log_count_kernel (hit-log counts), "
                      "HIP events on the launch stream",
            "peak_measured_stream_read": round(peak_meas, 1),
            "frac_of_measured": round(achieved / peak_meas, 4),
            "traffic_source": traffic_src,
        },
        "cpu_baseline": cpu,
        "gen_seconds": round(gen_s, 2),
    }
    if reduce_ms is not None:
        line["reduce_ms"] = round(reduce_ms, 3)
    if reduce_err is not None:
        line["reduce_error"] = reduce_err
    if host_path is not None:
        line["host_path"] = host_path
    if rank == 0:
        print(json.dumps(line), flush=True)
    if reduce_stuck:   # a stalled collective: do not wait on it in teardown
        sys.stdout.flush()
        os._exit(3)
    f.close()
    if dist is not None:
        dist.destroy_process_group()


def watched_reduce(fn, timeout):
    """The readout all-reduce on a watchdog thread (fn returns its ms):
    (ms, error, stuck) -- a failure or a stall is reported in the line,
    never keeps it from being printed, and a stall ends the rank with
    exit status 3 after the line (the per-CPU counter sum at readout,
    xdp-filter/xdp-filter.c:93-103)."""
    import threading
    box = {}

    def run():
        try:
            box["ms"] = fn()
        except Exception as e:  # reported, not fatal to the measurement
            box["err"] = repr(e)

    th = threading.Thread(target=run, daemon=True)
    th.start()
    th.join(timeout)
    stuck = th.is_alive()
    return box.get("ms"), ("timed out" if stuck else box.get("err")), stuck


def init_gloo():
    """The CPU process group (barriers, the max over ranks); gloo's connect
    message goes to stderr, so that stdout carries only the JSON line."""
    import torch.distributed as dist
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo")
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    return dist


def max_over_ranks(dist, wall):
    """The timed region's wall time, max over ranks (gloo; CPU tensor)."""
    if dist is None:
        return wall
    import torch
    t = torch.tensor([wall], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def stub_rank(args):
    """Launcher test body (no GPU): the rank's barriers and max-over-ranks
    wall time over gloo, the readout reduce on its watchdog (a gloo sum of
    the ranks' counter stand-ins in place of RCCL), and rank 0's line with
    n_gpus = world size, every rank's LOCAL_RANK (the device it would bind)
    and reduce_ms / reduce_error.  --stub-stall-rank R: rank R never
    finishes its timed region (the launcher's --rank-timeout kills the run);
    --stub-reduce-stall-rank R: rank R's reduce never completes."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if rank == args.stub_fail_rank:
        return 3
    dist = init_gloo() if world > 1 else None
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    if rank == args.stub_stall_rank:
        time.sleep(3600)
    if dist is not None:
        dist.barrier()
    wall = max_over_ranks(dist, time.perf_counter() - t1)
    locals_ = [local]
    reduce_ms, reduce_err, stuck = None, None, False
    if dist is not None:
        import torch
        locals_ = [None] * world
        dist.all_gather_object(locals_, local)

        def _reduce():
            if rank == args.stub_reduce_stall_rank:
                time.sleep(3600)
            t = torch.full((4,), rank + 1, dtype=torch.int64)
            tr = time.perf_counter()
            dist.all_reduce(t)
            if int(t[0]) != world * (world + 1) // 2:
                raise RuntimeError(f"reduce sum {int(t[0])}")
            return (time.perf_counter() - tr) * 1e3

        reduce_ms, reduce_err, stuck = watched_reduce(_reduce, args.reduce_timeout)
    if rank == 0:
        line = {"metric": METRIC, "value": 0.0, "unit": "Mpps", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(wall * 1e3 / max(args.steps, 1), 4),
                "local_ranks": locals_, "stub": True}
        if reduce_ms is not None:
            line["reduce_ms"] = round(reduce_ms, 3)
        if reduce_err is not None:
            line["reduce_error"] = reduce_err
        print(json.dumps(line), flush=True)
    if stuck:
        sys.stdout.flush()
        os._exit(3)
    if dist is not None:
        dist.destroy_process_group()
    return 0


def setup(args, rank, local):
    """Rules (1M IPv4 dst + 16 dst-port rules), the rank's C3 shard resident
    in HBM, and a dny_all context on device `local`."""
    import numpy as np
    import xftools as X
    import xfgpu as G
    n = 1 << args.log2_packets
    stride = 64
    # ---- rules: 1M IPv4 dst rules (seed 3) + 16 dst-port rules (tcp,udp)
    v4 = X.rand_keys(3, int(args.rules * 1.02) + 16, 4)[:args.rules]
    ports = (np.arange(16, dtype=np.uint16) * 1031 + 53).astype(np.uint16)
    # ---- traffic: C3 mix, shard seeded by rank
    t0 = time.time()
    data, lens = X.gen_workload(3 + 1000 * rank, 3, n, stride, v4=v4, ports=ports,
                                dst_permille=getattr(args, "dst_permille", 500),
                                port_permille=getattr(args, "port_permille", 250),
                                bad_permille=10)
    lens16 = lens.astype(np.uint16)
    gen_s = time.time() - t0

    f = G.Filter(G.FEAT_ALL | G.FEAT_DENY, devices=[local], ipv4_capacity=args.rules)
    assert f.prog_name == "xdpfilt_dny_all"
    f.update_batch(G.MAP_IPV4, v4, np.full(len(v4), 2, np.uint64))           # dst
    pkeys = np.array([X.port_key(int(p)) for p in ports], "<u4").view(np.uint8)
    f.update_batch(G.MAP_PORTS, pkeys, np.full(len(ports), 2 | 4 | 8, np.uint64))
    d_data = f.alloc(data.nbytes)
    d_data.upload(data)
    d_lens = f.alloc(lens16.nbytes)
    d_lens.upload(lens16)
    d_verd = f.alloc(n)
    del data

    alg_bytes = int(np.minimum(lens.astype(np.int64), 128).sum() + n)   # min(len,128)+1
    return f, (d_data, d_lens, d_verd), n, stride, lens, alg_bytes, v4, ports, gen_s



def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """The cores this process may use: its affinity set, capped by the
    pool's OMP_NUM_THREADS (a GPU box's CPU share; nproc shows the machine)."""
    t = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        t = min(t, int(omp))
    return max(t, 1)


def cpu_baseline(X, np, v4, ports, seconds):
    """The reference's CPU cost model on a 2^22-packet sample of the same C3
    workload (1M IPv4 rules): the C restatement of xdpfilt_dny_all with a
    hash index probed once per CHECK_MAP (BPF_MAP_TYPE_PERCPU_HASH,
    xdp-filter/xdpfilt_prog.h:56-64) and per-thread counters summed at the
    end, as per-CPU maps are (xdp-filter/xdp-filter.c:93-103) -- on every
    usable host core (`value`) and on one.  The parity checker's own rate
    (binary search over the sorted rules) is reported as `oracle_rate`
    only."""
    m = 1 << 22
    stride = 64
    buf = np.zeros(m * stride, np.uint8)
    lens = np.zeros(m, np.uint32)
    X.gen_workload(3, 3, m, stride, v4=v4, ports=ports, data=buf, lens=lens)
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 2, np.uint64)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    rules = rules.prepared()
    hmaps = X.OracleMaps(rules, hashed=True)
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]

    def rate(threads, secs, maps):
        done, t0 = 0, time.perf_counter()
        while True:
            X.run_oracle(feats, buf, lens, rules, stride=stride, maps=maps, nthreads=threads)
            done += m
            el = time.perf_counter() - t0
            if el >= secs:
                return done, el
    nt = host_threads()
    d1, e1 = rate(1, seconds * 0.4, hmaps)
    dn, en = rate(nt, seconds * 0.4, hmaps)
    do, eo = rate(1, seconds * 0.2, X.OracleMaps(rules))
    return {"value": round(dn / en / 1e6, 2), "unit": "Mpps", "cores": nt, "kind": "port",
            "value_1thread": round(d1 / e1 / 1e6, 2),
            "model": "C restatement of xdpfilt_dny_all (oracle/xf_oracle.c) with one hash "
                     "probe per CHECK_MAP (the BPF hash map's cost) and per-thread counters "
                     "summed at the end (per-CPU maps)",
            "oracle_rate_1thread": round(do / eo / 1e6, 2),
            "cpu_model": cpu_model(),
            "sample": f"2^22-packet C3 sample, 1M IPv4 rules: {dn // m} passes on {nt} threads "
                      f"({en:.1f}s), {d1 // m} on 1 thread ({e1:.1f}s); checker (binary "
                      f"search) {do // m} on 1 thread ({eo:.1f}s)",
            "c1": "not measured: the in-kernel XDP/veth run needs a BPF-capable clang, libbpf, "
                  "bpffs, iproute2 and root, absent from this image"}


if __name__ == "__main__":
    main()
