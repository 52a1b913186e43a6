"""The reference's shipped test-case input files (tests/golden/case_files.npz, packed by oracle/pack_case_files.py:
meshes and library tables, data only) unpacked into a directory, so the file-reading tests run without
/root/reference."""
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def unpack(dest, case):
    """Write case 'jet' (TURBOLENT_COMBUSTION) or 'plate' (TURBOLENT_FLAT_PLATE) files under dest; returns dest."""
    with np.load(os.path.join(GOLD, "case_files.npz")) as z:
        for key in z.files:
            c, rel = key.split("|", 1)
            if c != case:
                continue
            fn = os.path.join(dest, rel)
            os.makedirs(os.path.dirname(fn), exist_ok=True)
            with open(fn, "wb") as f:
                f.write(z[key].tobytes())
    return str(dest)
