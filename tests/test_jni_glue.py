"""CPU: the JNI glue a JVM backend binds (bindings/jni/gol_jni.c) stays in
step with include/gol.h and with its Scala declarations
(bindings/jni/GolNative.scala).  No JVM: the image has no JDK, so it compiles
with gcc -fsyntax-only -Werror against bindings/jni/jni_min/jni.h (a JNI
subset for this check only) -- a changed gol.h signature the glue calls breaks
this test; tests/test_gpu_jni_stub.py runs it on the GPU through a stub
JNIEnv."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "bindings", "jni")
GLUE = os.path.join(JNI, "gol_jni.c")
SCALA = os.path.join(JNI, "GolNative.scala")


def _compile(src_text=None, extra=()):
    cmd = ["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Wextra", "-Werror", "-pedantic",
           "-I" + os.path.join(JNI, "jni_min"), "-I" + os.path.join(ROOT, "include"), *extra]
    if src_text is None:
        return subprocess.run(cmd + [GLUE], capture_output=True, text=True)
    return subprocess.run(cmd + ["-x", "c", "-"], input=src_text, capture_output=True, text=True)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_glue_compiles_against_gol_h():
    r = _compile()
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_changed_gol_h_signature_breaks_the_glue(tmp_path):
    """The check has teeth: the same glue against a gol.h whose gol_step_ex
    lost its capacity argument does not compile."""
    inc = tmp_path / "include"
    inc.mkdir()
    hdr = open(os.path.join(ROOT, "include", "gol.h")).read()
    old = "int gol_step_ex(gol_ctx* ctx, uint32_t generations, uint64_t* hashes_out, size_t hashes_capacity);"
    assert old in hdr
    (inc / "gol.h").write_text(hdr.replace(old, "int gol_step_ex(gol_ctx* ctx, uint32_t generations, "
                                                "uint64_t* hashes_out);"))
    cmd = ["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Werror", "-I" + os.path.join(JNI, "jni_min"),
           "-I" + str(inc), GLUE]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode != 0 and "gol_step_ex" in r.stderr


def _c_entry_points():
    text = open(GLUE).read()
    return set(re.findall(r"Java_gameoflife_GolNative_(\w+)\s*\(", text))


def _scala_natives():
    text = open(SCALA).read()
    return set(re.findall(r"^\s*@native def (\w+)", text, re.M))


def test_every_native_method_has_its_entry_point():
    c, s = _c_entry_points(), _scala_natives()
    assert len(s) >= 25
    assert s == c, (s - c, c - s)


def test_arity_matches_scala_declarations():
    """JNI entry points take (JNIEnv*, jclass) plus the method's parameters."""
    text = open(GLUE).read()
    c_args = {}
    for m in re.finditer(r"Java_gameoflife_GolNative_(\w+)\s*\(([^)]*)\)", text):
        c_args[m.group(1)] = len([a for a in m.group(2).split(",") if a.strip()]) - 2
    scala = open(SCALA).read()
    for m in re.finditer(r"^\s*@native def (\w+)\(([^)]*)\)", scala, re.S | re.M):
        n = len([a for a in m.group(2).split(",") if a.strip()])
        assert c_args[m.group(1)] == n, m.group(1)


def test_glue_calls_only_declared_gol_entry_points():
    """Every gol_* function the glue calls is one include/gol.h declares (and
    so one libgol.so exports, tests/test_capi.py)."""
    from gameoflife import _native as N
    declared = set(N.header_symbols())
    called = set(re.findall(r"\b(gol_[a-z0-9_]+)\s*\(", open(GLUE).read()))
    assert called and called <= declared, called - declared


def test_integration_md_points_at_the_files():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "bindings/jni/gol_jni.c" in text and "bindings/jni/GolNative.scala" in text
    assert "Java_gameoflife_GolNative_create" not in text  # no second, hand-kept copy of the glue
