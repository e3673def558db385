"""Checkpoint format (include/vit_checkpoint.h) — host-only, runs on the CPU.

The reference's loader (train_vit.rs:89-143) reads a 256-int header and fp32 type-major params at
byte 1024; its save/load (:715-735) cover only `wte` without a header (D13), so there is no
reference-written file to pin against: the layout is checked here by an independent numpy
parser / writer against the library's C reader / writer, plus the error paths (bad magic,
truncation, config mismatch).
"""
import os

import numpy as np
import pytest

MAGIC, VERSION = 20261016, 1


def np_write(path, cfg, params, m=None, v=None, step=0, hp=(0, 0, 0, 0)):
    h = np.zeros(256, np.int32)
    n = params.size
    h[:14] = [MAGIC, VERSION, cfg.T, cfg.num_classes, cfg.num_layers, cfg.num_heads, cfg.channels,
              cfg.img, cfg.patch, cfg.in_ch, 1 if m is not None else 0, step, n & 0xFFFFFFFF, n >> 32]
    h[14:18] = np.array(hp, np.float32).view(np.int32)
    with open(path, "wb") as f:
        f.write(h.tobytes())
        f.write(np.asarray(params, np.float32).tobytes())
        if m is not None:
            f.write(np.asarray(m, np.float32).tobytes())
            f.write(np.asarray(v, np.float32).tobytes())


@pytest.fixture
def cfg(vit):
    return vit.data.CONFIGS["test"]


def test_num_params_matches_layout(vit):
    for name, cfg in vit.data.CONFIGS.items():
        assert vit.lib().vit_config_num_params(vit._cfg_c(cfg)) == cfg.num_params(), name


def test_library_writes_the_documented_layout(vit, cfg, tmp_path):
    rng = np.random.default_rng(0)
    n = cfg.num_params()
    p, m, v = (rng.standard_normal(n).astype(np.float32) for _ in range(3))
    path = tmp_path / "a.bin"
    vit.write_checkpoint(path, cfg, p, m, np.abs(v), step=7, adamw=(0.9, 0.95, 1e-8, 0.1))
    raw = path.read_bytes()
    assert len(raw) == 1024 + 3 * 4 * n
    h = np.frombuffer(raw[:1024], np.int32)
    assert list(h[:14]) == [MAGIC, VERSION, cfg.T, cfg.num_classes, cfg.num_layers, cfg.num_heads,
                            cfg.channels, cfg.img, cfg.patch, cfg.in_ch, 1, 7, n, 0]
    assert np.allclose(h[14:18].view(np.float32), [0.9, 0.95, 1e-8, 0.1])
    assert not h[18:].any()
    body = np.frombuffer(raw[1024:], np.float32)
    assert np.array_equal(body[:n], p) and np.array_equal(body[n:2 * n], m)
    assert np.array_equal(body[2 * n:], np.abs(v))
    assert not os.path.exists(str(path) + ".tmp")


def test_library_reads_numpy_written_file(vit, cfg, tmp_path):
    rng = np.random.default_rng(1)
    n = cfg.num_params()
    p = rng.standard_normal(n).astype(np.float32)
    path = tmp_path / "b.bin"
    np_write(path, cfg, p)
    info = vit.checkpoint_info(path)
    assert info["num_params"] == n and not info["has_opt"] and info["cfg"].T == cfg.T
    q, m, v = vit.read_checkpoint(path, cfg)
    assert np.array_equal(p, q) and m is None and v is None
    # with optimizer state
    m0, v0 = rng.standard_normal(n).astype(np.float32), rng.random(n).astype(np.float32)
    np_write(path, cfg, p, m0, v0, step=3, hp=(0.9, 0.999, 1e-8, 0.0))
    info = vit.checkpoint_info(path)
    assert info["has_opt"] and info["step"] == 3
    q, m, v = vit.read_checkpoint(path, cfg)
    assert np.array_equal(p, q) and np.array_equal(m, m0) and np.array_equal(v, v0)


def test_round_trip_through_the_parameter_split(vit, cfg, tmp_path):
    p = vit.data.init_params(cfg, "parity", seed=3)
    path = tmp_path / "c.bin"
    vit.write_checkpoint(path, cfg, p)
    q, _, _ = vit.read_checkpoint(path, cfg)
    for name, a in cfg.split(q).items():
        assert np.array_equal(a, cfg.split(p)[name]), name


@pytest.mark.parametrize("corrupt", ["magic", "truncated", "seq_len", "num_params", "extra_bytes"])
def test_rejects_bad_files(vit, cfg, tmp_path, corrupt):
    p = np.zeros(cfg.num_params(), np.float32)
    path = tmp_path / "d.bin"
    np_write(path, cfg, p)
    raw = bytearray(path.read_bytes())
    h = np.frombuffer(raw[:1024], np.int32).copy()
    if corrupt == "magic":
        h[0] = 20240326
    elif corrupt == "seq_len":
        h[2] += 1
    elif corrupt == "num_params":
        h[12] += 1
    raw[:1024] = h.tobytes()
    if corrupt == "truncated":
        raw = raw[:-4]
    elif corrupt == "extra_bytes":
        raw += b"\0" * 4
    path.write_bytes(bytes(raw))
    with pytest.raises(vit.VitError):
        vit.read_checkpoint(path, cfg)


def test_rejects_config_mismatch(vit, cfg, tmp_path):
    path = tmp_path / "e.bin"
    vit.write_checkpoint(path, cfg, np.zeros(cfg.num_params(), np.float32))
    other = vit.data.CONFIGS["test_t10"]
    with pytest.raises(vit.VitError):
        vit.read_checkpoint(path, other)
    with pytest.raises(vit.VitError):
        vit.checkpoint_info(tmp_path / "missing.bin")
