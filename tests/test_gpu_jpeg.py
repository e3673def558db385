"""GPU half of the JPEG input pipeline (jpeg.hip) through the C ABI, against Pillow's
libjpeg-turbo decode and the numpy restatement oracle/jpeg_ref.py (pinned to Pillow by
tests/test_jpeg_cpu.py): bit-exact uint8 output for every supported sampling kind, at identity
scale (the decoded pixels themselves) and through crops / flips / resizes; the trainer feed
(vit_trainer_set_batch_jpeg) gives the same loss and logits as uploading the oracle's pixels."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import jpeg_fixtures as jf  # noqa: E402
import jpeg_ref  # noqa: E402

pytestmark = pytest.mark.gpu


def _records(v, tmp_path, name, jpegs, labels=None):
    labels = np.arange(len(jpegs), dtype=np.int32) if labels is None else labels
    return v.write_jpeg_records(str(tmp_path / name), jpegs, labels)


def test_jpeg_identity_scale_equals_libjpeg_turbo(gpu, tmp_path):
    """Square images, centred box = the whole image, img = its size: the GPU's decoded pixels
    (IDCT, fancy upsampling, colour conversion) equal Pillow's, every byte, for 4:4:4, 4:2:2,
    4:2:0 and grayscale, optimised Huffman tables and restart intervals."""
    v = gpu
    for S in (224, 48):
        jpegs = [jf.encode(S, S, ss, q, kw, seed=S + i)
                 for i, (ss, q, kw) in enumerate([(0, 90, {}), (1, 85, {}), (2, 75, {"optimize": True}),
                                                  (-1, 95, {}), (2, 90, {"restart_marker_blocks": 5}),
                                                  (1, 60, {"restart_marker_rows": 2})])]
        L = v.JpegLoader(*_records(v, tmp_path, f"sq{S}", jpegs), batch=len(jpegs), shuffle=False, threads=3)
        lab, _, _ = L.next()
        out = L.decode_u8(S).numpy()
        for i, r in enumerate(lab):
            assert np.array_equal(out[i], jf.pil_rgb(jpegs[r])), (S, i)
        L.close()


@pytest.mark.parametrize("augment", [False, True])
def test_jpeg_crop_resize_matches_oracle(gpu, tmp_path, augment):
    """Mixed sizes and kinds (ImageNet-like 500x375 included), centred-square or random-resized
    crops with flips, resized to 224 and to 64: equal to jpeg_ref.resize of Pillow's decode with
    the loader's boxes, byte for byte, over two epochs."""
    v = gpu
    jpegs, labels = jf.dataset(12, seed=7)
    L = v.JpegLoader(*_records(v, tmp_path, "mix", jpegs, labels), batch=6, seed=3, shuffle=True,
                     augment=augment, threads=4)
    lab_to_rec = {int(l): i for i, l in enumerate(labels)}
    assert len(lab_to_rec) == len(labels)
    flips = 0
    for step in range(4):
        lab, ep, st = L.next()
        boxes = L.boxes()
        for img in (224, 64):
            out = L.decode_u8(img).numpy()
            for i, l in enumerate(lab):
                want = jpeg_ref.resize(jf.pil_rgb(jpegs[lab_to_rec[int(l)]]), boxes[i], img)
                assert np.array_equal(out[i], want), (step, i, boxes[i], img)
        flips += int(boxes[:, 4].sum())
    if augment:
        assert flips > 0
    L.close()


def test_jpeg_trainer_feed_matches_oracle_pixels(gpu, tmp_path):
    """vit_trainer_set_batch_jpeg (decode on the copy stream + device normalise) -> forward gives
    the loss and logits of forward() on the numpy-normalised oracle pixels, bit for bit, across the
    2-slot staging ring; labels come from the records."""
    v = gpu
    cfg = v.data.CONFIGS["test_h64"]
    B = 4
    jpegs, _ = jf.dataset(8, seed=11, sizes=((cfg.img, cfg.img), (40, 56), (75, 50)))
    labels = np.arange(8, dtype=np.int32)  # unique: the label names the record
    L = v.JpegLoader(*_records(v, tmp_path, "tr", jpegs, labels), batch=B, seed=2, shuffle=True,
                     augment=True, threads=2)
    params = v.data.init_params(cfg, "parity", seed=4)
    a = v.ViT.build(cfg, B, v.VIT_BF16, params=params)
    b = v.ViT.build(cfg, B, v.VIT_BF16, params=params)
    for step in range(5):
        lab, _, _ = L.next()
        boxes = L.boxes()
        a.set_batch_jpeg(L)
        la = a.forward()
        u8 = [jpeg_ref.resize(jf.pil_rgb(jpegs[int(l)]), boxes[i], cfg.img) for i, l in enumerate(lab)]
        px = jpeg_ref.normalise(np.stack(u8), v.IMAGENET_MEAN, v.IMAGENET_STD)
        lb = b.forward(px, lab)
        assert la == lb, (step, la, lb)
        assert np.array_equal(a.logits(), b.logits())
    a.close(); b.close(); L.close()


def test_jpeg_trainer_feed_rejects_batch_mismatch(gpu, tmp_path):
    """A loader opened with another batch size than the trainer's (e.g. the global batch instead of
    the per-rank one) is refused by vit_trainer_set_batch_jpeg before any pixel or label is copied
    (it would write past the trainer's staging buffer); the matching loader still feeds."""
    v = gpu
    cfg = v.data.CONFIGS["test_h64"]
    jpegs, _ = jf.dataset(8, seed=13, sizes=((cfg.img, cfg.img),))
    labels = np.arange(8, dtype=np.int32)
    m = v.ViT.build(cfg, 2, v.VIT_BF16, params=v.data.init_params(cfg, "parity", seed=4))
    for nb in (4, 1):
        L = v.JpegLoader(*_records(v, tmp_path, f"mm{nb}", jpegs, labels), batch=nb, shuffle=False, threads=1)
        L.next()
        with pytest.raises(v.VitError, match="trainer's batch is 2"):
            m.set_batch_jpeg(L)
        L.close()
    L = v.JpegLoader(*_records(v, tmp_path, "ok2", jpegs, labels), batch=2, shuffle=False, threads=1)
    L.next()
    m.set_batch_jpeg(L)
    assert np.isfinite(m.forward())
    L.close(); m.close()
