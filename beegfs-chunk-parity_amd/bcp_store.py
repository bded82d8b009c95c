"""Synthetic chunk stores for the loopback ranks.

Layout (one directory per storage target, as a BeeGFS storage target keeps
its chunk files, README.md of the reference):

    <root>/st<k>/chunks/<relative path>   chunk file of target k
    <root>/st<k>/parity/<relative path>   parity chunk file written by P

A work item is (path, timestamp, locations) with locations = chunk-holder
bitmask | P << 56 (common.h:19-25).
"""
from __future__ import annotations

import os
import time

import numpy as np

L_MASK = (1 << 56) - 1
NO_P = 0xFF


def with_p(locations: int, p: int) -> int:
    return (locations & L_MASK) | ((p & 0xFF) << 56)


def make_store(root: str, ntargets: int) -> str:
    for k in range(ntargets):
        os.makedirs(os.path.join(root, f"st{k}", "chunks"), exist_ok=True)
        os.makedirs(os.path.join(root, f"st{k}", "parity"), exist_ok=True)
    return root


def chunk_path(root: str, st: int, path: str) -> str:
    return os.path.join(root, f"st{st}", "chunks", path)


def parity_path(root: str, st: int, path: str) -> str:
    return os.path.join(root, f"st{st}", "parity", path)


def write_chunk(root: str, st: int, path: str, data) -> None:
    p = chunk_path(root, st, path)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "wb") as f:
        f.write(memoryview(np.ascontiguousarray(data, dtype=np.uint8)))


def read_file(p: str) -> bytes:
    with open(p, "rb") as f:
        return f.read()


def synthetic_chunk(seed: int, length: int) -> np.ndarray:
    """Uniform random bytes (numpy PCG64) for a chunk."""
    return np.random.default_rng(seed).integers(0, 256, size=length, dtype=np.uint8)


def random_layout(rng: np.random.Generator, ntargets: int, width: int) -> tuple[list[int], int]:
    """width chunk holders + one parity target outside them."""
    sts = rng.choice(ntargets, size=width + 1, replace=False)
    return sorted(int(x) for x in sts[:width]), int(sts[width])


def populate(root: str, ntargets: int, files, seed: int = 0, timestamp: int | None = None):
    """files: list of (path, holders, P, lengths).  Writes every chunk and
    returns (items, contents) with contents[path] = list of arrays in
    ascending holder order."""
    make_store(root, ntargets)
    ts = int(time.time()) + 3600 if timestamp is None else timestamp
    items, contents = [], {}
    for i, (path, holders, p, lengths) in enumerate(files):
        loc = 0
        arrs = []
        for h, L in zip(holders, lengths):
            data = synthetic_chunk(seed * 1_000_003 + i * 61 + h, L)
            write_chunk(root, h, path, data)
            loc |= 1 << h
            arrs.append(data)
        items.append((path, ts, with_p(loc, p)))
        contents[path] = arrs
    return items, contents
