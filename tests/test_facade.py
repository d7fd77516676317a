"""The reference-signature C++ facade (include/distributed_solver/instance.h):
a copy of the reference driver's call sequence (tests/cpp/reference_main.cpp)
compiles against it and prints the same topology as the reference binary."""
import os
import re
import subprocess

import pytest

from conftest import ROOT, load_golden

BIN = os.path.join(ROOT, "build", "reference_main")


@pytest.fixture(scope="module")
def driver():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "reference_main.cpp"),
                    "-L", os.path.join(ROOT, "distributedlpsolver_amd"), "-ldlp",
                    f"-Wl,-rpath,{os.path.join(ROOT, 'distributedlpsolver_amd')}", "-o", BIN],
                   check=True)
    return BIN


def test_topology_matches_reference_binary(driver):
    out = subprocess.run([driver, "1000", "1000", "0.1"], capture_output=True, text=True,
                         check=True).stdout
    ref = load_golden("ref_adalloc_1000.json")
    adv = [int(v) for v in re.findall(r"Advertiser \d+ degree is (\d+)", out)]
    imp = [int(v) for v in re.findall(r"Impression \d+ degree is (\d+)", out)]
    assert adv == ref["advertiser_degrees"] and imp == ref["impression_degrees"]
    assert out.startswith("Generated instance")


@pytest.mark.gpu
def test_reference_driver_solves_exactly(driver):
    out = subprocess.run([driver, "200", "200", "0.1", "solve"], capture_output=True, text=True,
                         check=True, timeout=300).stdout
    m = re.search(r"status (\d+) pivots (\d+) objective (\S+) revenue (\S+) max_infeasibility (\S+)",
                  out)
    assert m, out[-500:]
    rec = [r for r in load_golden("adalloc.json") if r["A"] == 200][0]
    assert int(m.group(1)) == 0
    assert abs(float(m.group(3)) - rec["highs_objective"]) <= 1e-9 * rec["highs_objective"]
    assert abs(float(m.group(4)) - float(m.group(3))) <= 1e-9 * float(m.group(3))
    assert float(m.group(5)) <= 1e-12
    assert "Dual Value = " in out
