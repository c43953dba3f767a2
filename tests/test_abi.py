"""CPU-side checks of the drop-in boundary: libg2048.so loads and exports every symbol that
include/g2048.h declares (no compute calls -- there is no GPU here)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "g2048.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"G2048_API\s+[\w\s\*]+?\b(g2048_\w+)\s*\(", src)))


def test_header_declares_abi():
    names = _declared()
    assert "g2048_env_step" in names and "g2048_replay_sample_encode" in names
    assert len(names) == 56


def test_library_exports_every_declared_symbol():
    import g2048._native as N

    lib = N.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert set(_declared()) == set(N.SIGNATURES)
    assert lib.g2048_abi_version() == 5
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = sorted(set(re.findall(r" T (g2048_\w+)", out)))
    assert exported == _declared()


def test_python_mirror_constants_match_header():
    """The Python host side lays out ReplayBuffer like g2048_replay_create: same section pad."""
    import g2048._native as N

    src = open(HEADER).read()
    pad = int(re.search(r"#define G2048_REPLAY_SECTION_PAD (\d+)", src).group(1))
    assert N.REPLAY_SECTION_PAD == pad and pad % 256 == 0 and pad % 4096 != 0
    assert int(re.search(r"#define G2048_ABI_VERSION (\d+)", src).group(1)) == N.ABI_VERSION


def test_no_cpu_fallback():
    """The product path fails loudly without a GPU instead of falling back."""
    import torch

    import g2048

    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    with pytest.raises(g2048.NativeError):
        g2048.VecEnv2048(16, device="cuda:0")
    with pytest.raises(g2048.NativeError):
        g2048.VecEnv2048(16, device="cpu")


def test_header_compiles_as_c():
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-x", "c", HEADER],
                   check=True)


def test_c_caller_compiles_and_links(tmp_path):
    """examples/abi_demo.c (a plain-C client) builds against the header and links libg2048.so;
    build() leaves the same binary in examples/ for tests/test_abi_gpu.py to run on the GPU."""
    import __graft_entry__ as G

    G.build_abi_demo(str(tmp_path / "abi_demo"))
    assert (tmp_path / "abi_demo").exists()


def test_entry_points_reject_bad_arguments():
    """Argument checks run before any device work: NULL / empty arguments come back as
    G2048_EINVAL with a message (here, without a GPU)."""
    import g2048._native as N

    lib = N.load()
    rc = lib.g2048_convnet_update(None, None, None, None, 8192, 0, None, 0.8, 1, None, None, None,
                                  None, None, None, None, 1e-2, 0.9, 0.999, 1e-8, 0, None)
    assert rc == N.G2048_EINVAL and b"convnet_update" in lib.g2048_last_error()
    rc = lib.g2048_convnet_forward_greedy(None, None, None, 0.5, 0.0, 0.0, None, None)
    assert rc == N.G2048_EINVAL and b"forward_greedy" in lib.g2048_last_error()
    rc = lib.g2048_convnet_targets(None, None, None, None, 0, 0, None, 0.8, 1, None, None, None)
    assert rc == N.G2048_EINVAL
    assert lib.g2048_convnet_train_workspace(0) == 0


def test_env_size_limit_refused_before_any_hip_call():
    """n > G2048_MAX_BOARDS (2^31 - 256: a grid stays below 2^32 work-items even where a board
    has two threads) is refused with G2048_EINVAL before the library touches a device, so this
    runs on the CPU."""
    import ctypes as C

    from g2048 import _native as N

    hdr = open(os.path.join(ROOT, "include", "g2048.h")).read()
    m = re.search(r"#define G2048_MAX_BOARDS \(\(int64_t\)(\d+)\)", hdr)
    assert m and int(m.group(1)) == (1 << 31) - 256 == N.MAX_BOARDS
    lib = N.load()
    out = C.c_void_p()
    rc = lib.g2048_env_create(C.byref(out), (1 << 31) - 255, 1, 0, 0, 0, None)
    assert rc == -1 and not out.value  # G2048_EINVAL
    assert b"G2048_MAX_BOARDS" in lib.g2048_last_error()


def test_vecenv_refuses_oversized_env_before_allocating():
    """VecEnv2048 checks n against G2048_MAX_BOARDS before it allocates or needs a GPU."""
    import g2048

    for n in (0, (1 << 31) - 255):
        with pytest.raises(ValueError, match="G2048_MAX_BOARDS"):
            g2048.VecEnv2048(n, device="cuda:0")
