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


def pytest_assertrepr_compare(config, op, left, right):
    """A failed == on large results (contig strings, link lists, dicts of 10^5+ entries) is
    reported by its first difference: pytest's own diff runs difflib over them for minutes,
    and a GPU run that prints nothing that long is taken for a hang."""
    sized = (list, tuple, bytes, str, dict)
    if op != "==" or not isinstance(left, sized) or not isinstance(right, sized):
        return None
    if max(len(left), len(right)) <= 200:
        return None
    a = list(left.items()) if isinstance(left, dict) else left
    b = list(right.items()) if isinstance(right, dict) else right
    i = next((j for j, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))
    show = lambda v: repr(v[i:i + 3])[:200]
    return ["%s of %d == %s of %d fails" % (type(left).__name__, len(left), type(right).__name__, len(right)),
            "first difference at index %d: %s != %s" % (i, show(a), show(b))]


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
