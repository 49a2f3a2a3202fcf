"""Achieved parity figures of the GPU tests (rel-L2, max-rel, PSNR, ...), not only their
pass / fail thresholds: every checker calls record(), and tests/conftest.py writes the
rows of the session to $C2D_PARITY_LOG (default gpurun_out/parity_metrics.tsv) at exit."""
import os

ROWS = []


def record(**metrics) -> None:
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    ROWS.append((test, {k: (float(v) if not isinstance(v, str) else v) for k, v in metrics.items()}))


def write(path) -> None:
    if not ROWS:
        return
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        for test, m in ROWS:
            f.write(test + "\t" + "\t".join(f"{k}={v:.4g}" if isinstance(v, float) else f"{k}={v}"
                                             for k, v in m.items()) + "\n")
