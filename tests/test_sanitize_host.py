"""The library's host C code under ASan + UBSan and under TSan (SURVEY.md §5:
level-ip's `make debug` is a -fsanitize=thread build, Makefile:17-18, and its
runner greps ThreadSanitizer reports, tests/test-run-all:41).

tests/sanitize/host_san.c drives level-ip_amd/csrc/csum_cpu.c (the per-call
drop-in, AVX-512, AVX2 and portable paths) and level-ip_amd/csrc/skb_batch.c (the frame
calls' multi-threaded host steps) against the oracle; see its header.
tests/sanitize/pool_san.cpp drives the host context's gather pool
(level-ip_amd/csrc/gather_pool.h) on its own.  tests/sanitize/frames_san.cpp
drives the host context and the host frame calls (csum_ctx.cpp,
frames_host.cpp: pieces, slots, the nontemporal gather, records, the apply
and its undo, registered regions, threads) over a CPU stand-in for the HIP
runtime and the device steps (tests/sanitize/hip_emu.cpp).  Host code only:
GPU sanitizers are not available on the MI355X pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, p) for p in (
    "level-ip_amd/csrc/csum_cpu.c", "level-ip_amd/csrc/skb_batch.c",
    "oracle/csum_oracle.c", "tests/sanitize/host_san.c")]
FLAGS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}
REPORTS = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer",
           "ERROR: LeakSanitizer")


def _build(kind, tmp_path):
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("gcc not available")
    exe = str(tmp_path / f"host_{kind}")
    r = subprocess.run([cc, "-O1", "-g", "-pthread", "-I", os.path.join(ROOT, "include"),
                        *FLAGS[kind], *SRCS, "-o", exe], capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr:
        pytest.skip(f"{kind} runtime not installed: {r.stderr.strip()[:200]}")
    assert r.returncode == 0, r.stderr
    return exe


def _check(r):
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert not [k for k in REPORTS if k in out], out[-4000:]
    assert "all checks passed" in r.stdout


@pytest.mark.parametrize("path", ["avx512", "avx2", "scalar"])
def test_host_code_asan_ubsan(tmp_path, path):
    exe = _build("asan", tmp_path)
    env = dict(os.environ, LVLIP_CPU_SUM=path)  # capped: the CPU may lack the wider ones
    _check(subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600))


def test_host_code_tsan(tmp_path):
    exe = _build("tsan", tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    if r.returncode != 0 and "unexpected memory mapping" in r.stderr:
        # gcc 11's TSan cannot place its shadow under some kernels' ASLR layout;
        # its documented remedy is to run with address randomisation off
        setarch = shutil.which("setarch")
        if setarch is None:
            pytest.skip("TSan needs ASLR off and setarch is absent")
        r = subprocess.run([setarch, os.uname().machine, "-R", exe],
                           capture_output=True, text=True, timeout=600)
    _check(r)


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_gather_pool(tmp_path, kind):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / f"pool_{kind}")
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-pthread",
                        "-I", os.path.join(ROOT, "level-ip_amd", "csrc"), *FLAGS[kind],
                        os.path.join(ROOT, "tests", "sanitize", "pool_san.cpp"), "-o", exe],
                       capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr:
        pytest.skip(f"{kind} runtime not installed: {r.stderr.strip()[:200]}")
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    if kind == "tsan" and r.returncode != 0 and "unexpected memory mapping" in r.stderr:
        setarch = shutil.which("setarch")
        if setarch is None:
            pytest.skip("TSan needs ASLR off and setarch is absent")
        r = subprocess.run([setarch, os.uname().machine, "-R", exe], capture_output=True, text=True,
                           timeout=300)
    _check(r)


FRAMES_C = [os.path.join(ROOT, p) for p in (
    "level-ip_amd/csrc/skb_batch.c", "level-ip_amd/csrc/csum_cpu.c", "oracle/csum_oracle.c")]
FRAMES_CXX = [os.path.join(ROOT, p) for p in (
    "level-ip_amd/csrc/frames_host.cpp", "level-ip_amd/csrc/csum_ctx.cpp",
    "tests/sanitize/hip_emu.cpp", "tests/sanitize/frames_san.cpp")]


def _build_frames(kind, tmp_path):
    cc, cxx = shutil.which("gcc"), shutil.which("g++")
    if cc is None or cxx is None:
        pytest.skip("gcc / g++ not available")
    if not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("HIP headers not available")
    inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "level-ip_amd", "csrc")]
    objs = []
    for src in FRAMES_C + FRAMES_CXX:
        obj = str(tmp_path / (os.path.basename(src) + f".{kind}.o"))
        if src.endswith(".c"):
            cmd = [cc, "-O1", "-g", "-pthread", *inc, *FLAGS[kind], "-c", src, "-o", obj]
        else:
            cmd = [cxx, "-std=c++17", "-O1", "-g", "-pthread", "-D__HIP_PLATFORM_AMD__",
                   "-I", "/opt/rocm/include", *inc, *FLAGS[kind], "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0 and "cannot find" in r.stderr:
            pytest.skip(f"{kind} runtime not installed: {r.stderr.strip()[:200]}")
        assert r.returncode == 0, r.stderr
        objs.append(obj)
    exe = str(tmp_path / f"frames_{kind}")
    r = subprocess.run([cxx, "-pthread", *FLAGS[kind], *objs, "-o", exe], capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr:
        pytest.skip(f"{kind} runtime not installed: {r.stderr.strip()[:200]}")
    assert r.returncode == 0, r.stderr
    return exe


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_frame_calls_sanitized(tmp_path, kind):
    exe = _build_frames(kind, tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    if kind == "tsan" and r.returncode != 0 and "unexpected memory mapping" in r.stderr:
        setarch = shutil.which("setarch")
        if setarch is None:
            pytest.skip("TSan needs ASLR off and setarch is absent")
        r = subprocess.run([setarch, os.uname().machine, "-R", exe], capture_output=True, text=True,
                           timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert not [k for k in REPORTS if k in out], out[-4000:]
    assert "frames_san: all checks passed" in r.stdout
