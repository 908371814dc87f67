"""examples/tx_rx_batch.c: INTEGRATION.md's TX/RX sketches as a plain C program
on the C ABI alone (built by __graft_entry__.build() / `make -C examples`).

On the GPU it fills the TCP and IPv4 checksums of 65 536 level-ip frames in one
call and checks every field against the per-call drop-in (tcp_v4_checksum's and
ip_send_check's arithmetic, src/tcp.c:87-103, src/ip_output.c:8-12), then
checks ip_rcv's verdicts for the same frames with every 97th one corrupted,
with the frames in malloc'd buffers and carved from one slab registered for
DMA or for zero-copy reads (INTEGRATION.md §2b'').  Without a GPU it must fail loudly: there is no CPU fallback behind the batch
calls."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "build", "tx_rx_batch")


def _exe():
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "examples")], check=True,
                       capture_output=True)
    return EXE


def test_example_fails_loudly_without_gpu():
    import lvlip

    if lvlip.device_count() > 0:
        pytest.skip("a GPU is present")
    r = subprocess.run([_exe(), "64"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no HIP device" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["malloc", "dma", "zerocopy"])
def test_example_tx_rx_batch(source):
    assert os.path.exists(EXE), "examples/build/tx_rx_batch not built (run __graft_entry__.build())"
    r = subprocess.run([EXE, "65536", source], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"tx_rx_batch ok: 65536 frames ({source})" in r.stdout, r.stdout


def test_example_rejects_unknown_source():
    r = subprocess.run([_exe(), "64", "pinned"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr, (r.returncode, r.stderr)


def test_install_and_build_against_it(tmp_path):
    """`make -C level-ip_amd install PREFIX=...` gives a level-ip build what it
    links: the example compiles and links against the
    installed headers and library alone."""
    prefix = tmp_path / "prefix"
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "level-ip_amd"), "install",
                    f"PREFIX={prefix}"], check=True, capture_output=True)
    for f in ("include/lvlip_csum.h", "include/lvlip_skb.h", "lib/liblvlip_csum.so"):
        assert (prefix / f).exists(), f
    exe = tmp_path / "tx_rx_batch"
    r = subprocess.run(["gcc", "-std=c99", "-D_POSIX_C_SOURCE=199309L", "-O2", "-Wall", "-Werror",
                        "-I", str(prefix / "include"), os.path.join(ROOT, "examples", "tx_rx_batch.c"),
                        "-L", str(prefix / "lib"), "-llvlip_csum", f"-Wl,-rpath,{prefix / 'lib'}",
                        "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run(["ldd", str(exe)], capture_output=True, text=True)
    assert str(prefix / "lib" / "liblvlip_csum.so") in r.stdout, r.stdout


MULTI = os.path.join(ROOT, "examples", "build", "multi_gpu")


def test_multi_gpu_example_fails_loudly_without_gpu():
    import lvlip

    if lvlip.device_count() > 0:
        pytest.skip("a GPU is present")
    _exe()
    r = subprocess.run([MULTI, "64", "2"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no HIP device" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("contexts", [2, 4])
def test_example_multi_gpu(contexts):
    """thread per context (on one GPU here: context k on
    device k % device_count), by the library and by hand with pthreads, every
    result against the per-call checksum()."""
    assert os.path.exists(MULTI), "examples/build/multi_gpu not built (run __graft_entry__.build())"
    r = subprocess.run([MULTI, "65536", str(contexts)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"over {contexts} contexts" in r.stdout, r.stdout
