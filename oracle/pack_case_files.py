"""Pack the input data files of the reference's two shipped test cases into tests/golden/case_files.npz, so the
next-4 tests (SU2 mesh reader, library readers, case_from_cfg, cfg -> device iteration) run where /root/reference
is absent (the GPU box). Data only: the meshes (SU2 ASCII), the mixture / chemistry / thermo / transport tables and
the library list files. The cfgs are not copied: the tests write theirs from oracle/make_golden.py's templates.

python oracle/pack_case_files.py   (needs /root/reference; test infrastructure)"""
import glob
import os

import numpy as np

REF = "/root/reference/Test_Cases/TURBOLENT"
CASES = {
    "jet": ("TURBOLENT_COMBUSTION",
            ["mesh_stretched.su2", "test_chem_second.txt", "test_chem_first.txt", "Mixture/Test_Mixture.txt",
             "Chemistry/Test_Reactions_second.txt", "Chemistry/Test_Reactions_first.txt", "Thermo/*.txt",
             "Transp/*.txt"]),
    "plate": ("TURBOLENT_FLAT_PLATE",
              ["mesh_flatplate_turb_137x97.su2", "test_air.txt", "Mixture/Test_Mixture_Air.txt",
               "Thermo/O2_thermo.txt", "Thermo/CO2_thermo.txt", "Thermo/N2_thermo.txt", "Transp/O2_transp.txt",
               "Transp/CO2_transp.txt", "Transp/N2_transp.txt"]),
}


def main():
    out = {}
    for case, (d, pats) in CASES.items():
        base = os.path.join(REF, d)
        for pat in pats:
            for fn in sorted(glob.glob(os.path.join(base, pat))):
                rel = os.path.relpath(fn, base)
                with open(fn, "rb") as f:
                    out[case + "|" + rel] = np.frombuffer(f.read(), dtype=np.uint8)
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                        "case_files.npz")
    np.savez_compressed(path, **out)
    print(f"{len(out)} files -> {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


if __name__ == "__main__":
    main()
