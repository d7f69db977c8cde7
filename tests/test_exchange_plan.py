"""CPU test (no GPU): the partitioned BFS's exchange arithmetic (csrc/exchange_plan.h), which RcclComm
and the native level loop use for the owner-routed pair exchange (the replacement of BfsSpark.java:90's
shuffle).  Compiled with g++ and run against a simulated send/recv transport and LocalGroupComm's pull
semantics on the same count tables (tests/cpp/test_exchange_plan.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exchange_plan_cpu(tmp_path):
    exe = tmp_path / "test_exchange_plan"
    src = os.path.join(ROOT, "tests", "cpp", "test_exchange_plan.cpp")
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-fsanitize=address,undefined", "-o", str(exe),
                    src], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True)
    assert "exchange plan ok" in out.stdout
