import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


def load_golden(name):
    with np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_names(prefix=""):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, prefix + "*.npz")))


def loop_case_flags(name):
    """Flags used by tests/golden/gen_golden.py for each loop_* case."""
    table = {
        "loop_tgass_preserve": ("TGASS", True, False),
        "loop_tgass_clip": ("TGASS", True, True),
        "loop_tgass_noconf": ("TGASS", True, False),
        "loop_tgass_nopreserve": ("TGASS", False, False),
        "loop_ass_preserve": ("ASS", True, False),
        "loop_tc_preserve": ("TC", True, True),
        "loop_as_preserve": ("AS", True, False),
        "loop_tgass_40x56": ("TGASS", True, False),
    }
    return table[name]


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture
def record_metric():
    """Append a measured parity number to gpurun_out/metrics.jsonl (merged back from the
    GPU box), so tolerances can be tightened from evidence."""
    import json
    import time

    def rec(name, value):
        d = os.path.join(ROOT, "gpurun_out")
        try:
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, "metrics.jsonl"), "a") as f:
                f.write(json.dumps({"name": name, "value": float(value), "time": time.time()}) + "\n")
        except OSError:
            pass
        print(f"[metric] {name} = {value:.3e}")
    return rec
