"""JPEG input pipeline, host half (no GPU): the entropy decoder + the numpy restatement of the
device half (oracle/jpeg_ref.py) against Pillow's libjpeg-turbo decode, bit for bit; header probe
and rejection of unsupported files; the record loader's sharding and crop boxes.

Pinning: the reference (ViT.rs) has no image decoder (its forward takes a prepared input array,
/root/reference/train_vit.rs:188); the oracle for decoded pixels is Pillow (libjpeg-turbo,
`PIL.features.version("jpg")`) run on the same files in this process."""
import io
import os
import sys

import numpy as np
import pytest
from PIL import Image

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import jpeg_fixtures as jf  # noqa: E402
import jpeg_ref  # noqa: E402


@pytest.mark.parametrize("h,w,ss,q,kw", jf.VARIANTS)
def test_host_decoder_and_oracle_match_libjpeg_turbo(vit, h, w, ss, q, kw):
    data = jf.encode(h, w, ss, q, kw, seed=h * w + q)
    W, H, kind = vit.jpeg_probe(data)
    assert (W, H) == (w, h)
    assert kind == {-1: 0, 0: 1, 1: 2, 2: 3}[ss]
    coef, info = vit.jpeg_coefficients(data)
    got = jpeg_ref.rgb_image(coef, info)
    assert np.array_equal(got, jf.pil_rgb(data))


def test_restart_markers_present(vit):
    data = jf.encode(64, 80, 2, 90, {"restart_marker_blocks": 3})
    assert b"\xff\xdd" in data and b"\xff\xd0" in data and b"\xff\xd1" in data


def test_unsupported_and_malformed_rejected(vit):
    b = io.BytesIO()
    jf.pixels(32, 32, False, 1).save(b, format="JPEG", progressive=True)
    with pytest.raises(vit.VitError, match="progressive"):
        vit.jpeg_coefficients(b.getvalue())
    b = io.BytesIO()
    jf.pixels(32, 32, False, 1).convert("CMYK").save(b, format="JPEG")
    with pytest.raises(vit.VitError, match="component"):
        vit.jpeg_probe(b.getvalue())
    with pytest.raises(vit.VitError, match="SOI"):
        vit.jpeg_probe(b"not a jpeg at all")
    good = jf.encode(32, 32, 2, 90, {})
    with pytest.raises(vit.VitError):
        vit.jpeg_coefficients(good[:40])


def test_resize_oracle_identity_and_flip():
    rgb = np.random.default_rng(0).integers(0, 256, size=(50, 50, 3)).astype(np.uint8)
    assert np.array_equal(jpeg_ref.resize(rgb, (0, 0, 50, 50, 0), 50), rgb)
    assert np.array_equal(jpeg_ref.resize(rgb, (0, 0, 50, 50, 1), 50), rgb[:, ::-1])
    # a 2x downscale of a crop averages 2x2 neighbourhoods at the half-pixel centres
    crop = jpeg_ref.resize(rgb, (10, 4, 40, 40, 0), 20)
    want = ((rgb[4:44:2, 10:50:2].astype(int) + rgb[5:44:2, 10:50:2] + rgb[4:44:2, 11:50:2] +
             rgb[5:44:2, 11:50:2]) * 16384 + 32768) >> 16
    assert np.array_equal(crop, want.astype(np.uint8))


def test_jpeg_loader_shards_and_boxes(vit, tmp_path):
    """Host half of the record loader (no GPU call): every rank of a 2-rank world sees the same
    number of steps and disjoint records of the epoch permutation (the uint8 loader's), labels
    follow the records, centred boxes are the largest centred square, augment boxes lie inside
    the image with aspect in [3/4, 4/3] and area >= 8 %, and are reproducible."""
    jpegs, labels = jf.dataset(24, seed=3)
    paths = vit.write_jpeg_records(str(tmp_path / "ds"), jpegs, labels)
    dims = [Image.open(io.BytesIO(j)).size for j in jpegs]
    lab_to_rec = {}
    for i, l in enumerate(labels):
        lab_to_rec.setdefault(int(l), []).append(i)
    seen = []
    for rank in range(2):
        L = vit.JpegLoader(*paths, batch=4, seed=9, rank=rank, world=2, shuffle=True, augment=False,
                               threads=2)
        assert L.steps_per_epoch == 3
        for _ in range(L.steps_per_epoch):
            lab, ep, st = L.next()
            boxes = L.boxes()
            for l, bx in zip(lab, boxes):
                cands = [r for r in lab_to_rec[int(l)] if (lambda W, H: min(W, H) == bx[2] == bx[3] and
                         bx[0] == (W - bx[2]) // 2 and bx[1] == (H - bx[3]) // 2)(*dims[r])]
                assert cands, (l, bx)
                assert bx[4] == 0
            seen += list(lab)
        L.close()
    assert sorted(seen) == sorted(labels.tolist())
    runs = []
    for _ in range(2):
        L = vit.JpegLoader(*paths, batch=8, seed=5, shuffle=True, augment=True, threads=3)
        L.next()
        runs.append(L.boxes())
        L.close()
    assert np.array_equal(runs[0], runs[1])
    b = runs[0]
    assert (b[:, 0] >= 0).all() and (b[:, 1] >= 0).all() and (b[:, 2] > 0).all() and (b[:, 3] > 0).all()
    assert set(b[:, 4].tolist()) <= {0, 1}


def test_jpeg_loader_reports_bad_record(vit, tmp_path):
    jpegs, labels = jf.dataset(4, seed=1)
    jpegs[2] = b"\xff\xd8garbage"
    paths = vit.write_jpeg_records(str(tmp_path / "bad"), jpegs, labels)
    L = vit.JpegLoader(*paths, batch=4, shuffle=False, threads=1)
    with pytest.raises(vit.VitError, match="image 2"):
        L.next()
    L.close()


def _segments(data):
    """(marker, start, end) of each marker segment up to and including the first SOS's entropy data"""
    out, p = [], 2
    while p < len(data) - 1:
        m = data[p + 1]
        n = int.from_bytes(data[p + 2:p + 4], "big")
        out.append((m, p, p + 2 + n))
        if m == 0xDA:
            e = p + 2 + n
            while not (data[e] == 0xFF and data[e + 1] not in (0x00,) and not 0xD0 <= data[e + 1] <= 0xD7):
                e += 1
            out[-1] = (m, p, e)
            break
        p += 2 + n
    return out


def test_second_frame_after_scan_rejected(vit):
    """SOI / SOF / SOS / SOF(larger) / SOS: a second frame header would resize the frame under scan
    buffers sized by the first; the parser must refuse it as libjpeg does."""
    small = jf.encode(16, 16, 0, 90, {})
    big = jf.encode(64, 96, 0, 90, {})
    segs = {m: (a, b) for m, a, b in _segments(big)}
    sof = big[segs[0xC0][0]:segs[0xC0][1]]
    sos = big[segs[0xDA][0]:segs[0xDA][1]]
    assert small.endswith(b"\xff\xd9")
    bad = small[:-2] + sof + sos + b"\xff\xd9"
    vit.jpeg_coefficients(small)  # the prefix itself decodes
    with pytest.raises(vit.VitError, match="duplicate SOF"):
        vit.jpeg_coefficients(bad)


def test_oversized_frame_rejected(vit):
    """A header of 65535 x 65535 pixels is refused before any allocation."""
    good = jf.encode(16, 16, 0, 90, {})
    (_, a, _), = [s for s in _segments(good) if s[0] == 0xC0]
    bad = bytearray(good)
    bad[a + 5:a + 9] = b"\xff\xff\xff\xff"   # height, width
    with pytest.raises(vit.VitError, match="too large"):
        vit.jpeg_probe(bytes(bad))
    with pytest.raises(vit.VitError, match="too large"):
        vit.jpeg_coefficients(bytes(bad))


@pytest.mark.timeout(120, method="thread")
def test_jpeg_loader_close_while_producing(vit, tmp_path):
    """Closing a loader while its producer is between batches (a pool job published, or about to
    be) must not deadlock: a job published before the stop runs to its end, none is published
    after it.  Many open / next / close cycles with the producer racing ahead (depth 3)."""
    jpegs, labels = jf.dataset(16, seed=7, sizes=((32, 32), (40, 24)))
    paths = vit.write_jpeg_records(str(tmp_path / "race"), jpegs, labels)
    for i in range(60):
        L = vit.JpegLoader(*paths, batch=[1, 2, 4][i % 3], shuffle=True, threads=1 + i % 3)
        if i % 2:
            L.next()
        L.close()
