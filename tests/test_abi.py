"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports every symbol that
include/eegnet_abi.h declares; host-side geometry/validation calls work without a GPU."""

from __future__ import annotations

import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "eegnet_abi.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(eegnet_\w+)\s*\(", txt, re.M)))


def test_header_matches_binding():
    from eegnetreplication_amd import _lib
    assert _header_symbols() == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_symbol():
    from eegnetreplication_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libeegnet_hip.so not built (run __graft_entry__.build())")
    lib = _lib.load()
    for name in _header_symbols():
        assert hasattr(lib, name), name
    assert b"gfx950" in lib.eegnet_build_info()
    txt = open(os.path.join(ROOT, "include", "eegnet_abi.h")).read()
    ver = int(re.search(r"#define EEGNET_ABI_VERSION (\d+)", txt).group(1))
    assert lib.eegnet_abi_version() == ver == _lib.ABI_VERSION


def test_param_count_and_validation():
    from eegnetreplication_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libeegnet_hip.so not built")
    d = _lib.dims(4096, 22, 256)
    assert _lib.param_count(d) == 1716          # paper Table 3 / SURVEY section 6
    assert _lib.workspace_bytes(d) > 4 * 4096 * 16 * 64 * 4
    d16 = _lib.dims(8, 64, 512, F1=16, D=4)
    assert _lib.param_count(d16) == 14116       # EEGNet-16,4 at 64x512
    with pytest.raises(RuntimeError, match="K1"):
        _lib.param_count(_lib.dims(8, 22, 256, K1=48))
    with pytest.raises(RuntimeError, match="F1\\*D"):
        _lib.param_count(_lib.dims(8, 22, 256, F1=3, D=1))


def test_shape_param_layout_matches_library():
    from eegnetreplication_amd import _lib
    from eegnetreplication_amd.ops import Shape
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libeegnet_hip.so not built")
    for C, T, F1, D in [(22, 256, 8, 2), (22, 257, 8, 2), (64, 512, 16, 4), (8, 64, 8, 2)]:
        s = Shape(C=C, T=T, F1=F1, D=D)
        assert s.n_params() == _lib.param_count(s.dims(4))


def _header_param_count(name):
    txt = open(os.path.join(ROOT, "include", "eegnet_abi.h")).read()
    m = re.search(r"^\s*(?:int|size_t|const char\*)\s+" + name + r"\s*\((.*?)\);", txt, re.S | re.M)
    args = m.group(1).strip()
    return 0 if args in ("", "void") else args.count(",") + 1


def test_binding_argument_counts_match_header():
    """Every ctypes signature has exactly as many arguments as the C prototype (a short argtypes
    list leaves trailing pointer arguments -- e.g. num_batches_tracked -- undefined)."""
    from eegnetreplication_amd import _lib
    for name, (_, args) in _lib._SIGS.items():
        assert len(args) == _header_param_count(name), name


def test_integration_ctypes_example_matches_binding():
    """The ctypes snippet a maintainer copies from INTEGRATION.md binds eegnet_train_step with the
    full parameter list (it once omitted num_batches_tracked) and passes every argument."""
    from eegnetreplication_amd import _lib
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"lib\.eegnet_train_step\.argtypes = \[(.*?)\]\n", txt, re.S)
    n_decl = m.group(1).count(",") + 1
    assert n_decl == len(_lib._SIGS["eegnet_train_step"][1]) == _header_param_count("eegnet_train_step")
    fields = re.findall(r'\("(\w+)", ctypes\.c_(?:int|float)\)', re.search(r"class Dims\(ctypes\.Structure\):(.*?)\]\n",
                                                                    txt, re.S).group(1))
    assert fields == [n for n, _ in _lib.Dims._fields_]          # the struct mirror, field for field
    call = re.search(r"rc = lib\.eegnet_train_step\((.*?)\)\s*(?:#.*)?\n(?=if rc)", txt, re.S).group(1)
    call = re.sub(r"#[^\n]*", "", call)
    depth, n_args = 0, 1
    for ch in call:
        depth += ch == "("
        depth -= ch == ")"
        n_args += ch == "," and depth == 0
    assert n_args == n_decl


def test_flag_and_kernel_id_constants_match_header():
    """The Python side's flag values and profiling kernel ids are the ones include/eegnet_abi.h
    documents (EEGNET_NO_CLAMP, EEGNET_KEY_FROM_STEP; eegnet_profile_enable's bit order)."""
    from eegnetreplication_amd import _lib, ops
    txt = open(os.path.join(ROOT, "include", "eegnet_abi.h")).read()
    flags = dict((k, int(v)) for k, v in re.findall(r"(EEGNET_[A-Z_]+)\s*=\s*(\d+)", txt))
    assert flags["EEGNET_NO_CLAMP"] == ops.NO_CLAMP
    assert flags["EEGNET_KEY_FROM_STEP"] == ops.KEY_FROM_STEP
    doc = re.search(r"i-th name eegnet_profile_collect reports:(.*?);", txt, re.S).group(1)
    assert [n.strip(" *\n") for n in doc.replace("\n", " ").split(",")] == list(_lib.KERNEL_IDS)


def test_cfg5_runs_the_compile_time_geometry_kernels():
    """The wide kernels compiled for EEGNet-16,4 at 64 x 512 (EEG_SHAPE_W5) are launched only when the
    run-time geometry equals the compiled one field for field; a layout change (coefficient block,
    workspace, LDS carve-up) that is not mirrored there would silently fall back to the generic
    kernels (cfg5 train 1.8M -> 1.4M trials/s).  No GPU needed."""
    import ctypes
    from eegnetreplication_amd import _lib
    lib = _lib.load()
    d5 = _lib.dims(1024, 64, 512, F1=16, D=4, K1=32)
    assert lib.eegnet_wide_spec(ctypes.byref(d5)) == 1, lib.eegnet_last_error().decode()
    for B in (1, 7, 4096):           # the batch is a run-time field
        d = _lib.dims(B, 64, 512, F1=16, D=4, K1=32)
        assert lib.eegnet_wide_spec(ctypes.byref(d)) == 1
    assert lib.eegnet_wide_spec(ctypes.byref(_lib.dims(4096, 22, 256))) == 0      # narrow
    assert lib.eegnet_wide_spec(ctypes.byref(_lib.dims(64, 64, 256, F1=16, D=4, K1=32))) == 0


def test_x_pitch_entry_point_and_validation():
    """eegnet_x_pitch: 260 for the recordings' 22 x 257 EEGNet-8,2 (16-byte rows), T elsewhere; a
    pitch is accepted only where the kernels honour it (checked by the geometry, no GPU needed)."""
    import ctypes
    from eegnetreplication_amd import _lib
    lib = _lib.load()
    xp = lambda *a, **k: lib.eegnet_x_pitch(ctypes.byref(_lib.dims(*a, **k)))
    assert xp(64, 22, 257) == 260
    assert xp(64, 22, 256) == 256
    assert xp(64, 22, 257, K1=64) == 257
    assert xp(64, 32, 257) == 257
    assert xp(64, 64, 512, F1=16, D=4) == 512
    nb = ctypes.c_size_t()
    ok = lambda d: lib.eegnet_workspace_bytes(ctypes.byref(d), ctypes.byref(nb))
    assert ok(_lib.dims(64, 22, 257, x_pitch=260)) == 0
    assert ok(_lib.dims(64, 22, 257, x_pitch=257)) == 0
    assert ok(_lib.dims(64, 22, 257, x_pitch=258)) != 0          # not a multiple of 4
    assert ok(_lib.dims(64, 22, 257, x_pitch=256)) != 0          # below T
    assert ok(_lib.dims(64, 32, 257, x_pitch=260)) != 0          # a runtime-shape kernel
    assert ok(_lib.dims(64, 22, 256, x_pitch=256)) == 0
    assert ok(_lib.dims(64, 22, 256, x_pitch=260)) != 0          # 22 x 256: pitch compiled in as T


def test_fold_mirror_matches_header():
    """The eegnet_fold mirror (_lib.Fold) and INTEGRATION.md's snippet list the header's fields in
    order (a field added to the struct -- xstat -- shifts every later one)."""
    from eegnetreplication_amd import _lib
    txt = open(os.path.join(ROOT, "include", "eegnet_abi.h")).read()
    body = re.search(r"typedef struct eegnet_fold \{(.*?)\} eegnet_fold;", txt, re.S).group(1)
    fields = re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(\w+);", body, re.M)
    assert fields == [n for n, _ in _lib.Fold._fields_]
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    snippet = re.search(r"class Fold\(ctypes\.Structure\):(.*?)\nassert", doc, re.S).group(1)
    assert re.findall(r'"(\w+)"', snippet) == fields


def test_x_stats_width_matches_pass_a_row_head():
    """eegnet_x_stats_width = K1 + 1 + the edge items (head pairs, tail pairs, head and tail sums):
    pass A's partial-row head a fold launch with xstat replaces."""
    import ctypes
    from eegnetreplication_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libeegnet_hip.so not built")
    lib = _lib.load()
    for K1 in (32, 64):
        P, R = (K1 - 1) // 2, K1 - 1 - (K1 - 1) // 2
        want = K1 + 1 + R * (R + 1) // 2 + P * (P + 1) // 2 + R + P
        assert lib.eegnet_x_stats_width(ctypes.byref(_lib.dims(64, 22, 257, K1=K1))) == want
    assert lib.eegnet_x_stats_width(ctypes.byref(_lib.dims(64, 64, 512, F1=16, D=4))) < 0    # narrow path only


def test_retired_persist_flag_is_rejected():
    """Round 5's opt-in one-launch persistent step (flag bit 4) is gone from the shipped library: the
    C-ABI rejects that bit (and every other unknown one) before any launch, so no caller -- FusedTrainer,
    DataParallelTrainer, FoldBatch or a C binding -- can reach a step whose results are not the
    five-launch step's bit for bit.  Runs without a GPU: the flag check precedes every device call."""
    import ctypes
    import inspect
    from eegnetreplication_amd import _lib, ops
    from eegnetreplication_amd.model import FusedTrainer
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libeegnet_hip.so not built")
    assert "persist" not in inspect.signature(FusedTrainer).parameters
    assert "persist" not in inspect.signature(ops.train_step).parameters
    assert not hasattr(ops, "PERSIST")
    lib = _lib.load()
    d = _lib.dims(64, 22, 256)
    dummy = ctypes.c_void_p(256)                     # never dereferenced: the call fails on the flags
    for flags in (4, 4 | 2, 8, 1 << 20):
        rc = lib.eegnet_train_step(ctypes.byref(d), dummy, dummy, dummy, dummy, 1, 2, dummy, dummy, dummy,
                                   1e-3, 0.9, 0.999, 1e-7, dummy, None, dummy, None, flags, None)
        assert rc == -1, flags
        assert b"unknown flags" in lib.eegnet_last_error()
    hdr = open(os.path.join(ROOT, "include", "eegnet_abi.h")).read()
    assert "EEGNET_PERSIST" not in hdr
