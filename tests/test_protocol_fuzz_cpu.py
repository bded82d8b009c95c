"""The protocol's random rounds (tests/test_gpu_protocol_fuzz.py) on the CPU:
the P role's fold is the test double (tests/native/cpu_xor_hook.c), so this
checks the host logic -- lanes, both P-role folds, both wires, the fold
service width, window replay, missing chunks, rebuild lanes, and ranks as
threads (loopback) or as processes (socketpairs) -- against the oracle on
machines without a GPU.  The batched pipeline needs the device and is left to
the GPU test."""
import os

from test_gpu_protocol_fuzz import fuzz_rounds


def test_random_rounds_with_the_cpu_fold(bcp, oracle, tmp_path, cpu_hook):
    fuzz_rounds(bcp, oracle, tmp_path, float(os.environ.get("BCP_FUZZ_SECONDS", "5")),
                int(os.environ.get("BCP_FUZZ_SEED", "11")), ("pipelined", "batched", "procs"))
