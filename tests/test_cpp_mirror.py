"""Run the C++ restatement of packet/acl_internal_test.go (tests/cpp/) that
drives libnffacl through the C++ host mirror nff-go_amd/host/nffgo.hpp."""
import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "tests" / "cpp" / "acl_internal_test"


@pytest.fixture(scope="module")
def binary():
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "cpp")], check=True)
    return BIN


def _run(binary, which):
    env = dict(os.environ, NFFACL_GOLDEN=str(ROOT / "tests" / "golden"))
    r = subprocess.run([str(binary), which], capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "--- FAIL" not in r.stdout
    return r.stdout


def test_cpp_parse_tests(binary):
    out = _run(binary, "parse")
    for name in ("TestGetL3ACLFromTextTable", "TestGetL3ACLFromJSON", "TestGetL3ACLErrors",
                 "TestGetL2ACLFromJSON", "TestGetL2ACLFromTextTable"):
        assert f"--- PASS: {name}" in out, out


@pytest.mark.gpu
def test_cpp_match_tests(binary):
    out = _run(binary, "match")
    for name in ("TestInternal_l4ACL_packetIPv4_TCP", "TestInternal_l3ACL_packetIPv4_TCP",
                 "TestInternal_l3ACL_l4ACL_packetIPv4_TCP", "TestInternal_l3ACL_l4ACL_packetIPv6_TCP",
                 "TestInternal_l3ACL_l4ACL_packetIPv6_UDP", "TestInternal_l3ACL_l4ACL_packetIPv4_ICMP",
                 "TestInternal_l3ACL_l4ACL_packetIPv6_ICMP", "TestVectorSeparatorStability",
                 "TestInternal_l2ACL_packetIPv4", "TestInternal_l2ACL_packetARP",
                 "TestVectorSeparatorSharedBatcher", "TestScalarSeparatorService", "TestRuleReloadStep08"):
        assert f"--- PASS: {name}" in out, out
