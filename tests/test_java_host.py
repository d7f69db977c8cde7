"""CPU checks of the Java host (java/), which this image cannot compile (no JDK):

* java/bfsx_jni.c compiles with -Werror against include/bfsx.h and a minimal JNI header written from the JNI
  specification (tests/jni_stub/jni.h): a forward whose call drifts from the C-ABI (a renamed entry point, a
  changed argument list) fails here;
* every `native` method of Bfsx.java has its JNI forward in bfsx_jni.c and every forward has its method;
* the Java sources use no API newer than Java 7, the reference's source level (pom.xml:16 `<source>1.7`;
  round 3 used Java 8's Math.toIntExact).
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

JAVA = os.path.join(ROOT, "java")
SRC = os.path.join(JAVA, "it", "unitn", "bd", "bfs")


def _strip_comments(text):
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    return re.sub(r'"(?:\\.|[^"\\])*"', '""', text)  # string literals (log messages) are not code


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_jni_forwards_compile_against_the_c_abi():
    cmd = ["gcc", "-fsyntax-only", "-std=c99", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
           "-Werror=implicit-function-declaration", "-I", os.path.join(ROOT, "tests", "jni_stub"),
           "-I", os.path.join(ROOT, "include"), os.path.join(JAVA, "bfsx_jni.c")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_native_methods_match_jni_forwards():
    java = _strip_comments(open(os.path.join(SRC, "Bfsx.java")).read())
    natives = set(re.findall(r"\bnative\s+[\w\[\]]+\s+(\w+)\s*\(", java))
    c = open(os.path.join(JAVA, "bfsx_jni.c")).read()
    forwards = set(re.findall(r"\bJava_it_unitn_bd_bfs_Bfsx_(\w+)\s*\(", c))
    assert natives, "no native methods found"
    assert natives == forwards, (sorted(natives - forwards), sorted(forwards - natives))


# Java 8+ library calls and syntax (lambdas, method references) a Java 7 compiler rejects
JAVA8 = [r"\bMath\.(?:toIntExact|addExact|subtractExact|multiplyExact|floorMod|floorDiv)\b", r"\.stream\(\)",
         r"\bString\.join\b", r"\bjava\.util\.function\b", r"\bjava\.util\.Optional\b", r"\bjava\.time\b",
         r"\.forEach\(", r"\.getOrDefault\(", r"\.computeIfAbsent\(", r"\.removeIf\(", r"\bStandardCharsets\.\w+\.name",
         r"\)\s*->", r"\b\w+\s*->\s*[\w{(]", r"\w::\w", r"\bvar\s+\w+\s*="]


@pytest.mark.parametrize("name", ["Bfsx.java", "BfsGpu.java"])
def test_java_sources_are_java7(name):
    text = _strip_comments(open(os.path.join(SRC, name)).read())
    hits = [(p, m.group(0)) for p in JAVA8 for m in re.finditer(p, text)]
    assert not hits, f"{name} uses APIs or syntax newer than Java 7: {hits}"


def test_java_host_options_devices_and_dump_levels():
    """BfsGpu honours `devices` (N ranks through Bfsx.initGroup, the group context of
    bfsx_init_group) and `dumpLevels` (every pass's problemFile_k, BfsSpark.java:115-116), each from a system
    property or the service.properties key, as the C++ twin does."""
    text = _strip_comments(open(os.path.join(SRC, "BfsGpu.java")).read())
    raw = open(os.path.join(SRC, "BfsGpu.java")).read()
    assert re.search(r'option\("devices",\s*"1"\)', raw) and "Bfsx.initGroup(" in text
    assert re.search(r'option\("dumpLevels",\s*"false"\)', raw)
    # inside the per-pass loop: every pass written when dumpLevels, the last pass always
    assert re.search(r"if\s*\(dumpLevels\s*\|\|\s*k\s*==\s*passes\)\s*write\(", text)
    # GRAY for the vertices a pass discovered (d == pass), WHITE beyond it
    assert "d == pass ? Color.GRAY : Color.BLACK" in raw and "d > pass" in raw
