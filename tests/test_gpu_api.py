"""GPU: the reference's own tests (pubsub_test.go: TestBasicPubsub,
TestNodesDropping, TestLowerNodesDropping, TestNodesDroppingGracefully) plus
a paced 1000-message run, a burst, two topics, the wire codec and
INTEGRATION.md's cgo shim sequence over more than two message windows, written
against the C++ mirror of the reference API (include/pubsub.hpp) and run as
one native binary (tests/cpp/pubsub_test.cpp) whose floods go through
libpsengine.so on the GPU.  Same skip sets and assertions as the reference.
"""
import subprocess

import pytest

from psengine import _build

pytestmark = pytest.mark.gpu

TESTS = ["TestWireCodec", "TestBasicPubsub", "TestNodesDropping", "TestLowerNodesDropping",
         "TestNodesDroppingGracefully", "TestPaced1000", "TestBurstOrder", "TestTwoTopics", "TestShimWindowFlush"]


@pytest.fixture(scope="module")
def results():
    exe = _build.build_cpp_tests()
    p = subprocess.run([exe], capture_output=True, text=True, timeout=200)
    return p.returncode, p.stdout + p.stderr


@pytest.mark.parametrize("name", TESTS)
def test_reference_api_test(results, name):
    rc, out = results
    assert f"--- PASS: {name}" in out, out
