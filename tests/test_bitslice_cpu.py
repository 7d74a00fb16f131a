"""The bitsliced RS(12,8) encode A/B (tools/tune/gen_bitslice.py, measured in
profiles/r05/rs12_cauchy_ab.txt F): its XOR network, evaluated on the CPU, equals
the byte-wise GF(2^8) products of ISA-L's Cauchy parity rows, and the committed
network (tools/tune/bitslice_net.inc) is the one the generator writes."""
import os
import subprocess
import sys

from tests.conftest import ROOT


def test_generator_self_check_and_committed_network():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tune", "gen_bitslice.py")], capture_output=True,
                       text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]  # the generator asserts 2,000 random columns against GF products
    assert "chosen: karatsuba" in r.stderr
    with open(os.path.join(ROOT, "tools", "tune", "bitslice_net.inc")) as f:
        assert f.read() == r.stdout
