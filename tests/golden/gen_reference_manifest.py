"""Record the reference's own golden streams as a SHA-256 manifest (run in the build container only).

Sources (read-only, not copied): /root/reference/sw/tests/data/compressed_2d_<n>.zfp and
/root/reference/hw/tests/data/compressed_2d_<n>.zfp -- headerless zfp streams of the 2-D Gaussian bump
(sw/tests/test_zfp.cpp:13-25) at tolerance 1e-3 (test_zfp.cpp:72-73). The 530/550/590/600 goldens were made
from inputs whose x*x + y*y was summed in float32; `recipe` records which generator reproduces each.
The first and last stream words are kept so a mismatch can be localised without the files.
"""
import hashlib
import json
import os

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    out = []
    for sub in ("sw/tests/data", "hw/tests/data"):
        d = os.path.join(REF, sub)
        for f in sorted(os.listdir(d)):
            if not (f.startswith("compressed_2d_") and f.endswith(".zfp")):
                continue
            n = int(f[len("compressed_2d_"):-4])
            b = open(os.path.join(d, f), "rb").read()
            w = np.frombuffer(b, dtype=np.uint64)
            out.append(dict(file="%s/%s" % (sub, f), n=n, tolerance=1e-3,
                            recipe="bump_f32sum" if n in (530, 550, 590, 600) else "bump",
                            bytes=len(b), sha256=hashlib.sha256(b).hexdigest(),
                            first_words=[int(x) for x in w[:3]], last_word=int(w[-1])))
    with open(os.path.join(HERE, "reference_goldens.json"), "w") as fp:
        json.dump(dict(source="fpgasystems/gcow goldens (sha256 manifest; files not copied)",
                       script="tests/golden/gen_reference_manifest.py", goldens=out), fp, indent=1)
    print(len(out), "goldens")


if __name__ == "__main__":
    main()
