"""Randomised descriptor batches through bcp_xor_stripes against the oracle,
for a time budget (BCP_FUZZ_SECONDS, default 8 s; a longer soak is the same
test with a larger budget).  Each round draws a batch -- widths 1..56, lengths
from 0 B to 4 MiB (tiny, unaligned, exact 16-byte multiples, tile-sized),
misaligned sources and outputs, missing sources, rebuild truncation
(out_len below the longest source), window replay (quirk A3-q1) -- and the
engine's tuning (tile sizes of both kernels, the argument form on or off,
tables read from host or device memory), so every path of the engine takes
part: xor_stream's pointer-table form for uniform batches, xor_desc_args for
small ones, desc_tiles + xor_desc / xor_desc_p for the rest, including the
grouped, wide and general tile paths.  Every output byte is compared with
the oracle (window replay: the parity body of oracle.gen_parity_file, the
reference's algorithm restated; otherwise the zero-padded XOR)."""
import os
import time

import numpy as np
import pytest

from test_gpu_xor import Dev, gpu_stripes  # noqa: F401  (helpers of the device tests)

pytestmark = pytest.mark.gpu
KiB, MiB = 1024, 1024 * 1024
TUNING = {  # engine option -> values drawn per round (the first is the default)
    "vecs_per_thread": [0, 1, 2, 4, 8],
    "desc_vecs_per_thread": [0, 1, 2, 4, 8, 16],
    "desc_args_max": [16, 0, 4],
    "table_host_max": [4096, 0, 1 << 24],
    "desc_table_host_max": [128 * 1024, 0, 1 << 24],
}


def _length(rng, big):
    r = rng.random()
    if r < 0.15:
        return int(rng.integers(0, 48))                      # tiny, zero included
    if r < 0.35:
        return 16 * int(rng.integers(1, 4097))               # 16-byte multiples up to 64 KiB
    if r < 0.55:
        return 32 * KiB * int(rng.integers(1, 9))            # whole tiles
    return int(rng.integers(1, big + 1))                     # anything (unaligned)


def _batch(rng, budget_bytes):
    """A list of stripe dicts for gpu_stripes and their expected outputs."""
    from oracle import gen_parity_file, xor_padded_np
    stripes, refs, used = [], [], 0
    uniform = rng.random() < 0.2
    nstripes = int(rng.integers(1, 41))
    width = int(rng.choice([1, 2, 3, 4, 5, 8, 9, 12, 16, 24, 56], p=[.08, .1, .1, .1, .08, .24, .06, .08, .08, .04, .04]))
    ulen = 16 * int(rng.integers(1, 32 * KiB)) if uniform else 0
    for _ in range(nstripes):
        n = width if uniform or rng.random() < 0.6 else int(rng.integers(1, 57))
        big = 4 * MiB if n <= 8 else 512 * KiB
        lens = [ulen if uniform else _length(rng, big) for _ in range(n)]
        if used + sum(lens) > budget_bytes and stripes:
            break
        used += sum(lens)
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
        if not uniform and n > 1 and rng.random() < 0.1:
            chunks[int(rng.integers(0, n))] = None           # a missing source (length 0)
        m = max((0 if c is None else len(c)) for c in chunks)
        st = dict(chunks=chunks, out_len=m)
        window = 0
        if not uniform and m > 64 * KiB and rng.random() < 0.15:
            # window replay: a window below the longest source (a multiple of 16)
            window = 16 * int(rng.integers(1024, m // 16))
            st["window"] = window
        elif not uniform and m and rng.random() < 0.2:
            st["out_len"] = int(rng.integers(1, m + 1))       # rebuild truncation
        if not uniform:
            st["pads"] = [int(x) for x in rng.integers(0, 16, size=n)]
            st["dst_pad"] = int(rng.integers(0, 16))
        present = [np.zeros(0, np.uint8) if c is None else c for c in chunks]
        if window:
            body = np.frombuffer(gen_parity_file(present, window), dtype=np.uint8)[8 * n:]
        else:
            body = xor_padded_np(present)
        ref = np.zeros(st["out_len"], np.uint8)
        k = min(len(body), st["out_len"])
        ref[:k] = body[:k]
        stripes.append(st)
        refs.append(ref)
    return stripes, refs


def test_random_batches_match_the_oracle(oracle, engine, queue):
    budget = float(os.environ.get("BCP_FUZZ_SECONDS", "8"))
    seed = int(os.environ.get("BCP_FUZZ_SEED", "2026"))
    rng = np.random.default_rng(seed)
    defaults = {k: engine.option(k) for k in TUNING}
    t_end = time.monotonic() + budget
    rounds = stripes_done = bytes_done = 0
    forms = set()
    try:
        while time.monotonic() < t_end or rounds < 3:
            tuning = {k: (v[0] if rng.random() < 0.5 else v[int(rng.integers(0, len(v)))]) for k, v in TUNING.items()}
            for k, v in tuning.items():
                engine.option(k, v)
            stripes, refs = _batch(rng, 48 * MiB)
            dev = Dev(engine, queue)
            try:
                outs = gpu_stripes(dev, queue, stripes)
            finally:
                dev.free()
            forms.add(engine.option("last_desc_form"))
            for i, (o, r) in enumerate(zip(outs, refs)):
                if not np.array_equal(o, r):
                    bad = np.flatnonzero(o != r)
                    st = stripes[i]
                    lens = [0 if c is None else len(c) for c in st["chunks"]]
                    pytest.fail(f"seed {seed} round {rounds} stripe {i}: {bad.size} bytes differ from {bad[0]}; "
                                f"lens {lens} out_len {st['out_len']} window {st.get('window', 0)} "
                                f"pads {st.get('pads')} dst_pad {st.get('dst_pad', 0)} tuning {tuning}")
            rounds += 1
            stripes_done += len(stripes)
            bytes_done += sum(len(r) for r in refs)
            if rounds % 50 == 0:
                print(f"fuzz: {rounds} batches ...", flush=True)  # progress for long soaks
    finally:
        for k, v in defaults.items():
            engine.option(k, v)
    print(f"fuzz: {rounds} batches, {stripes_done} stripes, {bytes_done / MiB:.1f} MiB of output, "
          f"descriptor forms seen {sorted(forms)}")
    assert rounds >= 3
