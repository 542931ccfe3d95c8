"""pytest configuration: `gpu` marker, import paths for the product package
(pycuda-euler_amd/, reference-style top-level modules) and the test-only oracle."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pycuda-euler_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)

# the library's test / diagnostic overrides (EULERHIP_NO_SK2, EULERHIP_FORCE_FILTER, ...) take
# effect only with EULERHIP_DEBUG set (csrc/common.h Knobs)
os.environ.setdefault("EULERHIP_DEBUG", "1")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def golden_cases(*names, alphabet="acgtn"):
    out = []
    for n in names:
        for c in load_golden(n)["cases"]:
            ext = c["name"].startswith("extended")
            if (alphabet == "acgtn" and not ext) or (alphabet == "extended" and ext) or alphabet == "all":
                out.append(c)
    return out


@pytest.fixture(scope="session")
def gpu_session():
    import eulerhip
    s = eulerhip.Session(0)
    yield s
    s.close()
