"""Regenerates tests/golden/kats.json.

KAT-1..KAT-4 are the known answers SURVEY.md §8(c) records from the UNCHANGED
reference task_processing.c (built and run in the survey container); they are
copied here as data and are what pins the oracle.  The "edge" vectors are
produced by the oracle restatement (oracle/bcp_oracle.c) once it reproduces
all four KATs, so they are regression vectors for the GPU path (n in
{1,2,3,5,8} x lengths {1,7,8,9,15,16,17,4095,65536} as §8(c) asks, plus
mixed-length stripes).  xor_parity inputs are the KAT-1 generator; gen_file
inputs are the splitmix64 stream oracle.synthetic(len, seed=1000+k) (the KAT
chunk generator makes every chunk's byte j identical, which cancels).  Each
fixture stores only lengths and SHA-256 of the expected output.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

SURVEY_KATS = {
    "KAT-1": {"kind": "xor_parity", "n": 8, "s": 524288,
              "sha256": "07854d2fef297a06ba81685e660c332de36d5d18d546927d30daad6d7fda1541",
              "fnv1a64": "0feb61957bfd0383"},
    "KAT-2": {"kind": "gen_file", "lens": [524288] * 8, "file_len": 524352, "rebuild_victim": 3,
              "sha256": "dbd07ee2e0bc2c102cd4bd46840930de586b0e36822a33d1ba516ece5192f0d3"},
    "KAT-3": {"kind": "gen_file", "lens": [65536, 4194304, 524288, 3145745, 1, 200000, 4194304, 65536],
              "file_len": 4194368, "rebuild_victim": 1,
              "sha256": "54ed1f904264185344498e410c7b1770b79516bc7b5ab17716d41b8e65e4ce09"},
    "KAT-4": {"kind": "gen_file", "lens": [10485760, 26214405], "file_len": 26214421, "rebuild_victim": 0,
              "sha256": "0115cfb16da88ba3c11fc591cd6ee07886bc603ff571a2b593c87fd80bfa2021"},
}


def edge_vectors():
    out = []
    for n in (1, 2, 3, 5, 8):
        for L in (1, 7, 8, 9, 15, 16, 17, 4095, 65536):
            data = O.kat1_data(n, L)
            par = O.xor_parity(data, L, n)
            out.append({"kind": "xor_parity", "n": n, "s": L, "sha256": hashlib.sha256(par.tobytes()).hexdigest()})
    mixed = [[1, 7], [0, 17, 16], [4095, 4096, 4097, 1], [65536, 0, 65521, 12345, 99999],
             [3, 200000, 17, 65536, 1, 0, 8, 131073]]
    for lens in mixed:
        chunks = [O.synthetic(L, 1000 + k) for k, L in enumerate(lens)]
        pf = O.gen_parity_file(chunks)
        out.append({"kind": "gen_file", "lens": lens, "file_len": len(pf),
                    "sha256": hashlib.sha256(pf).hexdigest()})
    # small-window replay (A3-q1) cases: window 4096 bytes, multi-window streams
    for lens in ([4096, 10000], [5000, 12288, 1], [8192, 4096, 16385]):
        chunks = [O.synthetic(L, 1000 + k) for k, L in enumerate(lens)]
        pf = O.gen_parity_file(chunks, window=4096)
        out.append({"kind": "gen_file", "lens": lens, "window": 4096, "file_len": len(pf),
                    "sha256": hashlib.sha256(pf).hexdigest()})
    return out


def main():
    doc = {"_source": __doc__.strip().splitlines()[0], "survey_kats": SURVEY_KATS, "edge": edge_vectors()}
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
