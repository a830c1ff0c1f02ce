"""The Cycles Device plugin (integration/device_hip.cpp) compiles against the
reference headers, and every C-ABI call it makes is declared in
include/hipcycles.h."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
LIB = os.path.join(REF, "lib", "linux_centos7_x86_64")


def test_plugin_uses_only_declared_entry_points():
    src = open(os.path.join(ROOT, "integration", "device_hip.cpp")).read()
    hdr = open(os.path.join(ROOT, "include", "hipcycles.h")).read()
    used = set(re.findall(r"\b(hipcy_[a-z_0-9]+)\s*\(", src))
    declared = set(re.findall(r"\b(hipcy_[a-z_0-9]+)\s*\(", hdr))
    used -= {"hipcy_init", "hipcy_create_device"}  # none expected; guard against typos
    assert used and used <= declared, used - declared


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "blender", "intern", "cycles")) or not shutil.which("g++"),
                    reason="reference tree not present")
def test_plugin_compiles_against_reference_headers():
    cyc = os.path.join(REF, "blender", "intern", "cycles")
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-DCCL_NAMESPACE_BEGIN=namespace ccl {", "-DCCL_NAMESPACE_END=}",
           "-I" + cyc, "-I" + os.path.join(LIB, "tbb", "include"), "-I" + os.path.join(LIB, "openimageio", "include"),
           "-I" + os.path.join(LIB, "openexr", "include"), "-I" + os.path.join(LIB, "boost", "include"),
           "-I" + os.path.join(REF, "blender", "intern", "atomic"),
           "-I" + os.path.join(REF, "blender", "intern", "guardedalloc"),
           "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "integration", "device_hip.cpp")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
