"""Regenerates tests/golden/ref_xor.json from the REFERENCE'S OWN xor_parity.

Container only: needs oracle/_ref/libref_xor.so, which oracle/Makefile `ref`
compiles from /root/reference/src/beegfs-raid5/common/task_processing.c:96-109
unchanged (the function needs no MPI).  The fixtures are data: lengths, seeds
and SHA-256 values (hex outputs for the tiny cases) -- no reference text.

Inputs are distinct rows of the splitmix64 byte stream (oracle.synthetic, the
same stream libbcp's bcp_dev_fill_synthetic writes on the device): row k of a
case is synthetic(len, seed + k), rows contiguous as xor_parity's `data`
([nsources][nbytes], task_processing.c:206).  input_sha256 pins the generator.

  kind "xor_parity": out = ref_xor_parity(rows, len, n)
      n in {1,2,3,5,8,13,56} x len in {1,7,8,9,15,16,17,4095,65536,524288,524289}
  kind "gen_file":  a parity chunk file whose every fold is ref_xor_parity; the
      window assembly around it (zero padding after a short read, replay of
      the last window past EOF, header, truncation) is chunk_sender /
      parity_generator (task_processing.c:163-226, 282-308) restated here,
      because those roles need MPI and cannot be built.  KAT-3's and KAT-4's
      lengths with distinct per-chunk data (the survey KATs' generator makes
      every chunk's bytes identical, so its parity bodies cancel).

    make -C oracle ref && python tests/golden/make_ref_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

W = O.WINDOW
XOR_NS = (1, 2, 3, 5, 8, 13, 56)
XOR_LENS = (1, 7, 8, 9, 15, 16, 17, 4095, 65536, 524288, 524289)
GEN_CASES = [
    {"name": "KAT-3-distinct", "lens": [65536, 4194304, 524288, 3145745, 1, 200000, 4194304, 65536],
     "seed": 3000, "rebuild_victim": 1},
    {"name": "KAT-4-distinct", "lens": [10485760, 26214405], "seed": 4000, "rebuild_victim": 0},
    {"name": "mixed-odd", "lens": [3, 200000, 17, 65536, 1, 9, 8, 131073], "seed": 5000, "rebuild_victim": 7},
    {"name": "config2-stripe", "lens": [524288] * 8, "seed": 6000, "rebuild_victim": 3},
]


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def rows(n: int, length: int, seed: int) -> np.ndarray:
    return np.concatenate([O.synthetic(length, seed + k) for k in range(n)]) if length else np.zeros(0, np.uint8)


def case_seed(n: int, length: int) -> int:
    return 1_000_000 + 1000 * n + XOR_LENS.index(length)


def windows_fold(sources, max_cs: int) -> np.ndarray:
    """parity_generator's window loop over chunk_sender streams, each fold
    done by the reference's xor_parity.  sources: byte arrays (file bytes)."""
    n = len(sources)
    buffer_size = min(W, max_cs)
    expected = -(-max_cs // W)
    bufs = [np.zeros(buffer_size, np.uint8) for _ in range(n)]
    pos = [0] * n
    sent = [0] * n
    out = np.zeros(max_cs, np.uint8)
    left, off = max_cs, 0
    for _ in range(expected):
        for k, src in enumerate(sources):
            data_left = max_cs - sent[k]
            if sent[k] < len(src):  # refill only while the file has bytes (A3-q1)
                r = min(buffer_size, data_left, len(src) - pos[k])
                bufs[k][:r] = src[pos[k]:pos[k] + r]
                pos[k] += r
                bufs[k][r:] = 0
            sent[k] += buffer_size
        blk = O.ref_xor_parity(np.concatenate(bufs), buffer_size, n)
        w = min(buffer_size, left)
        out[off:off + w] = blk[:w]
        off += w
        left -= w
    return out


def gen_case(c):
    lens, seed = c["lens"], c["seed"]
    chunks = [O.synthetic(L, seed + k) for k, L in enumerate(lens)]
    max_cs = max(lens)
    body = windows_fold(chunks, max_cs)
    pf = np.concatenate([np.array(lens, dtype="<u8").view(np.uint8), body])
    v = c["rebuild_victim"]
    survivors = [ch for k, ch in enumerate(chunks) if k != v] + [body]
    rebuilt = windows_fold(survivors, max_cs)[:lens[v]]
    assert sha(rebuilt) == sha(chunks[v]), "reference fold does not round-trip"
    return {"kind": "gen_file", "name": c["name"], "lens": lens, "seed": seed, "file_len": int(pf.size),
            "sha256": sha(pf), "rebuild_victim": v, "rebuilt_sha256": sha(rebuilt),
            "inputs_sha256": [sha(ch) for ch in chunks]}


def main():
    if O.build_ref() is None or O.ref_lib() is None:
        sys.exit("oracle/_ref/libref_xor.so not built (needs /root/reference)")
    cases = []
    for n in XOR_NS:
        for L in XOR_LENS:
            seed = case_seed(n, L)
            data = rows(n, L, seed)
            out = O.ref_xor_parity(data, L, n)
            fx = {"kind": "xor_parity", "n": n, "len": L, "seed": seed,
                  "input_sha256": sha(data), "sha256": sha(out)}
            if L <= 64:
                fx["out_hex"] = out.tobytes().hex()
            cases.append(fx)
    for c in GEN_CASES:
        cases.append(gen_case(c))
    doc = {"_source": "reference xor_parity (task_processing.c:96-109, sha256 of its text "
                      "086856bd7d9eb27fab974f0d6f391a9393a3081d9426e5be482e431c6482137f) "
                      "compiled unchanged by oracle/Makefile `ref`; see tests/golden/make_ref_golden.py",
           "window": W, "cases": cases}
    with open(os.path.join(HERE, "ref_xor.json"), "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(f"{len(cases)} fixtures")


if __name__ == "__main__":
    main()
