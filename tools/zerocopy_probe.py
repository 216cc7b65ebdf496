#!/usr/bin/env python3
"""tools/zerocopy_probe.py — what the classify kernel sustains reading its
frames straight from pinned, mapped host memory over PCIe (diagnostic, not
the product path): C3 (64 B frames at a 64 B stride) and C5 (1514 B frames
at a 1536 B stride, 64-byte header windows) batches in host memory,
registered with hipHostRegisterMapped, their device addresses passed to
xfg_classify_timed as a device-resident batch would be; lengths and
verdicts in HBM.  Prints one JSON line per case: frames/s and the PCIe
bytes the windows stand for."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))
import numpy as np  # noqa: E402
import xftools as X  # noqa: E402
import xfgpu as G  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]


def mapped(arr):
    rc = hip.hipHostRegister(arr.ctypes.data, arr.nbytes, 2 | 1)   # Mapped | Portable
    assert rc == 0, rc
    p = C.c_void_p()
    rc = hip.hipHostGetDevicePointer(C.byref(p), arr.ctypes.data, 0)
    assert rc == 0, rc
    return p.value


def case(name, kind, n, stride, n4, n6, nports, iters=5):
    v4 = X.rand_keys(kind, int(n4 * 1.02) + 16, 4)[:n4]
    v6 = X.rand_keys(kind + 100, int(n6 * 1.02) + 16, 16)[:n6] if n6 else None
    ports = (np.arange(nports, dtype=np.uint32) * 61 + 53).astype(np.uint16)
    data, lens = X.gen_workload(kind, kind, n, stride, v4=v4, v6=v6, ports=ports)
    f = G.Filter(G.FEAT_ALL | G.FEAT_DENY, devices=[0], ipv4_capacity=n4, ipv6_capacity=max(n6, 1024))
    f.update_batch(G.MAP_IPV4, v4, np.full(len(v4), 2, np.uint64))
    if n6:
        f.update_batch(G.MAP_IPV6, v6, np.full(len(v6), 2, np.uint64))
    pk = np.array([X.port_key(int(p)) for p in ports], "<u4").view(np.uint8)
    f.update_batch(G.MAP_PORTS, pk, np.full(len(ports), 2 | 4 | 8, np.uint64))
    lens16 = lens.astype(np.uint16)
    d_lens, d_verd = f.alloc(lens16.nbytes), f.alloc(n)
    d_lens.upload(lens16)
    hptr = mapped(data)
    f.classify_timed(hptr, d_lens.ptr, n, stride, d_verd.ptr, 1, lens_u16=True)
    ms = f.classify_timed(hptr, d_lens.ptr, n, stride, d_verd.ptr, iters, lens_u16=True)
    win = min(stride, 64)
    # the same batch resident in HBM, for the verdicts' check and the ratio
    d_data = f.alloc(data.nbytes)
    d_data.upload(data)
    v_host = np.zeros(n, np.uint8)
    d_verd.download(v_host)
    ms_dev = f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_verd.ptr, iters, lens_u16=True)
    v_dev = np.zeros(n, np.uint8)
    d_verd.download(v_dev)
    hip.hipHostUnregister(data.ctypes.data)
    print(json.dumps({"case": name, "packets": n, "stride": stride, "path": f.last_path(),
                      "zero_copy_ms": round(ms, 3), "Mpps": round(n / ms / 1e3, 1),
                      "window_GBps": round(n * win / ms / 1e6, 1),
                      "device_resident_ms": round(ms_dev, 3),
                      "verdicts_equal": bool(np.array_equal(v_host, v_dev))}), flush=True)
    f.close()


def c5_mix(n=1 << 22, stride=1536, reps=4):
    """Do the kernel's zero-copy reads and the DMA engines' strided copies of
    header windows add up?  Half a C5 batch classified in place while the
    other half's windows go by hipMemcpy2DAsync (64 and 128 bytes a row),
    each alone and then both at once in two threads."""
    import threading
    import time
    kind, n4, n6, nports = 5, 15_000_000, 1_000_000, 1024
    v4 = X.rand_keys(kind, int(n4 * 1.02) + 16, 4)[:n4]
    v6 = X.rand_keys(kind + 100, int(n6 * 1.02) + 16, 16)[:n6]
    ports = (np.arange(nports, dtype=np.uint32) * 61 + 53).astype(np.uint16)
    data, lens = X.gen_workload(kind, kind, n, stride, v4=v4, v6=v6, ports=ports)
    f = G.Filter(G.FEAT_ALL | G.FEAT_DENY, devices=[0], ipv4_capacity=n4, ipv6_capacity=n6)
    f.update_batch(G.MAP_IPV4, v4, np.full(len(v4), 2, np.uint64))
    f.update_batch(G.MAP_IPV6, v6, np.full(len(v6), 2, np.uint64))
    half = n // 2
    lens16 = lens[:half].astype(np.uint16)
    d_lens, d_verd = f.alloc(lens16.nbytes), f.alloc(half)
    d_lens.upload(lens16)
    hptr = mapped(data)
    d_win = f.alloc(half * 128)
    hip.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipMemcpy2DAsync.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t,
                                     C.c_size_t, C.c_int, C.c_void_p]
    hip.hipStreamSynchronize.argtypes = [C.c_void_p]
    st = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(st)) == 0
    src = data.ctypes.data + half * stride
    out = {}

    def zc():
        t0 = time.perf_counter()
        f.classify_timed(hptr, d_lens.ptr, half, stride, d_verd.ptr, reps, lens_u16=True)
        out["zc"] = half * reps / (time.perf_counter() - t0) / 1e6

    def dma(w):
        def run():
            t0 = time.perf_counter()
            for _ in range(reps):
                assert hip.hipMemcpy2DAsync(d_win.ptr, w, src, stride, w, half, 1, st) == 0
                assert hip.hipStreamSynchronize(st) == 0
            out[f"dma{w}"] = half * reps / (time.perf_counter() - t0) / 1e6
        return run

    zc()
    for w in (64, 128):
        dma(w)()
    alone = dict(out)
    for w in (64, 128):
        out.clear()
        ta, tb = threading.Thread(target=zc), threading.Thread(target=dma(w))
        ta.start(); tb.start(); ta.join(); tb.join()
        print(json.dumps({"case": f"c5_mix_{w}", "Mpps_alone": {k: round(v, 1) for k, v in alone.items()},
                          "Mpps_together": {k: round(v, 1) for k, v in out.items()},
                          "sum_together": round(sum(out.values()), 1)}), flush=True)
    hip.hipHostUnregister(data.ctypes.data)
    f.close()


if __name__ == "__main__":
    if sys.argv[1:] == ["mix"]:
        c5_mix()
    else:
        case("c3", 3, 1 << 22, 64, 1_000_000, 0, 16)
        case("c5", 5, 1 << 21, 1536, 15_000_000, 1_000_000, 1024)
