#!/usr/bin/env python3
"""Generate tests/golden/xdpfilter_golden.npz: the regression fixture.

Runs the ten programs of the CPU restatement (oracle/xf_oracle.c) over:
  * every known-answer frame of tests/kat.py (SURVEY.md Appendix A and the
    behaviours of xdp-filter/tests/test-xdp-filter.sh / test_basic.py) with
    the rule set kat_rules();
  * a seeded structured-fuzz corpus (tools/xfsynth.c) with a random rule set;
and stores inputs + expected outputs (verdicts, rule values after the run,
per-action stats) as plain arrays.  The fixture is data only; regenerate with
`make oracle && python tests/golden/make_golden.py`.

Provenance: round 1 generated these same arrays from the reference's
xdpfilt_*.c compiled for the host against stand-in BPF headers; such a build
is not a reference build by this project's rules (the reference needs
libbpf's headers and the kernel's map runtime, absent here: DESIGN.md §2),
so it was removed and the fixture is now what the restatement produces
(byte-identical to the round-1 file until round 3 added the reference-traffic
rows Q1-Q20 to tests/kat.py).  It is RESTATEMENT-DERIVED: it pins regressions
of the restatement and of the HIP path, not parity with the reference; the
reference-held expectations are tests/kat.py's rows.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.dirname(HERE))

import xftools as X  # noqa: E402
import kat  # noqa: E402

STRIDE = 160
N_FUZZ = 6000


def pack(frames, stride):
    data = np.zeros(len(frames) * stride, np.uint8)
    lens = np.zeros(len(frames), np.uint32)
    for i, f in enumerate(frames):
        assert len(f) <= stride, len(f)
        data[i * stride:i * stride + len(f)] = np.frombuffer(f, np.uint8)
        lens[i] = len(f)
    return data, lens


def rules_arrays(prefix, rs: X.RuleSet, out):
    nz = np.nonzero(rs.ports)[0]
    out[prefix + "port_idx"] = nz.astype(np.uint32)
    out[prefix + "port_vals"] = rs.ports[nz]
    for name in ("v4_keys", "v4_vals", "v6_keys", "v6_vals", "eth_keys", "eth_vals"):
        out[prefix + name] = getattr(rs, name)


def main():
    out = {}
    # ---- known-answer corpus
    kf = kat.kat_frames()
    kdata, klens = pack([f for _, f, _ in kf], STRIDE)
    krules = kat.kat_rules()
    out["kat_data"], out["kat_lens"] = kdata, klens
    out["kat_names"] = np.array([n for n, _, _ in kf])
    rules_arrays("kat_rules_", krules, out)
    # ---- fuzz corpus
    frules, pool = X.random_rules(2024, n4=48, n6=24, ne=12, nports=20)
    fdata, flens = X.gen_fuzz(77, N_FUZZ, STRIDE, frules, pool)
    out["fuzz_data"], out["fuzz_lens"] = fdata, flens
    rules_arrays("fuzz_rules_", frules, out)
    out["stride"] = np.array(STRIDE)

    for v, feats in X.VARIANTS:
        for tag, data, lens, rs in (("kat", kdata, klens, krules), ("fuzz", fdata, flens, frules)):
            verd, after, st = X.run_oracle(feats, data, lens, rs, stride=STRIDE)
            p = f"{tag}_{v}_"
            out[p + "verdicts"] = verd
            nz = np.nonzero(rs.ports | after.ports)[0]
            out[p + "port_idx"] = nz.astype(np.uint32)
            out[p + "port_vals"] = after.ports[nz]
            out[p + "v4_vals"] = after.v4_vals
            out[p + "v6_vals"] = after.v6_vals
            out[p + "eth_vals"] = after.eth_vals
            out[p + "stats"] = st
    path = os.path.join(HERE, "xdpfilter_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path)} bytes): {len(kf)} KAT frames, {N_FUZZ} fuzz frames")


if __name__ == "__main__":
    main()
