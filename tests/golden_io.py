"""Loader for the committed golden fixtures under tests/golden/ (data only)."""
import json
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"


def load_golden(name):
    p = GOLDEN / f"{name}.npz"
    if p.exists():
        with np.load(p, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    return json.loads((GOLDEN / f"{name}.json").read_text())
