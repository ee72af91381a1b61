"""GPU: the C ABI driven from a plain C program (tests/c_abi/c_abi_rollout.c) with no Python or
torch in the process -- reset, fused rollouts across MT19937 reset events, a single step and
the final state at N = 5, 100 (no goal) and 1,500, bit for bit against the C oracle -- and the
ABI's error contract.  The binary is built on the CPU by __graft_entry__.build()."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_abi", "c_abi_rollout")


def test_c_host_program_bit_exact():
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} not built (run __graft_entry__.build())")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "C ABI: OK" in r.stdout, r.stdout
    assert r.stdout.count("bit-exact vs the C oracle: yes") == 3, r.stdout
