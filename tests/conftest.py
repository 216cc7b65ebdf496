import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "xdp-tools_amd", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


GOLDEN = os.path.join(ROOT, "tests", "golden", "xdpfilter_golden.npz")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return np.load(GOLDEN, allow_pickle=False)


def golden_rules(g, prefix):
    import numpy as np
    import xftools as X
    rs = X.RuleSet()
    rs.ports[g[prefix + "port_idx"]] = g[prefix + "port_vals"]
    for name in ("v4_keys", "v4_vals", "v6_keys", "v6_vals", "eth_keys", "eth_vals"):
        setattr(rs, name, np.array(g[prefix + name]))
    return rs


def golden_expected_ports(g, prefix, base):
    out = base.ports.copy()
    out[g[prefix + "port_idx"]] = g[prefix + "port_vals"]
    return out
