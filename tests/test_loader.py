"""Input pipeline host side (include/vit_data.h) — CPU only (pinned = 0 makes
no HIP call).  The native loader's batches are checked record by record against the numpy
mirror of its documented order (data.epoch_permutation / loader_batch_records): seeded
per-epoch shuffle, disjoint rank shards, dropped partial global batch, file order without
shuffle; plus the file-size checks."""
import numpy as np
import pytest


def make_files(tmp_path, n, img, seed=0):
    rng = np.random.default_rng(seed)
    imgs = rng.integers(0, 256, size=(n, img, img, 3), dtype=np.uint8)
    labs = rng.integers(0, 1000, size=n, dtype=np.int32)
    ip, lp = tmp_path / "img.u8", tmp_path / "lab.i32"
    imgs.tofile(ip)
    labs.tofile(lp)
    return imgs, labs, ip, lp


@pytest.mark.parametrize("world,shuffle", [(1, True), (2, True), (3, False)])
def test_loader_batches_follow_the_documented_order(vit, tmp_path, world, shuffle):
    n, img, B, seed = 37, 8, 4, 99
    imgs, labs, ip, lp = make_files(tmp_path, n, img)
    steps = n // (B * world)
    seen = {}
    for rank in range(world):
        ld = vit.Loader(ip, lp, img, B, seed=seed, rank=rank, world=world, shuffle=shuffle,
                        pinned=False, depth=2)
        assert ld.num_records == n and ld.steps_per_epoch == steps
        for seq in range(2 * steps + 1):  # two epochs and into the third
            x, y, ep, st = ld.next()
            ids, ep_r, st_r = vit.data.loader_batch_records(n, B, world, rank, seed, seq, shuffle)
            assert (ep, st) == (ep_r, st_r)
            assert np.array_equal(x, imgs[ids]) and np.array_equal(y, labs[ids])
            seen.setdefault(ep, []).extend(ids.tolist())
        ld.close()
    for ep in (0, 1):  # ranks are disjoint within an epoch and cover world*B*steps records
        ids = seen[ep]
        assert len(ids) == len(set(ids)) == world * B * steps
    if shuffle:
        assert vit.data.epoch_permutation(n, seed, 0).tolist() != vit.data.epoch_permutation(n, seed, 1).tolist()
    else:
        assert seen[0][:B] == list(range(B))


def test_permutation_is_a_permutation(vit):
    for n in (1, 2, 5, 64):
        p = vit.data.epoch_permutation(n, 7, 3)
        assert sorted(p.tolist()) == list(range(n))


def test_loader_rejects_bad_files(vit, tmp_path):
    imgs, labs, ip, lp = make_files(tmp_path, 10, 8)
    with pytest.raises(vit.VitError):
        vit.Loader(ip, lp, 9, 2, pinned=False)  # record size mismatch
    with pytest.raises(vit.VitError):
        vit.Loader(ip, lp, 8, 11, pinned=False)  # fewer records than one batch
    with pytest.raises(vit.VitError):
        vit.Loader(tmp_path / "missing", lp, 8, 2, pinned=False)


def test_normalize_mirror(vit):
    x = np.arange(2 * 2 * 2 * 3, dtype=np.uint8).reshape(2, 2, 2, 3) * 10
    y = vit.data.normalize_u8(x, (0.5, 0.4, 0.3), (0.2, 0.25, 0.5))
    assert y.shape == (2, 3, 2, 2) and y.dtype == np.float32
    assert y[1, 2, 1, 0] == np.float32((np.float32(x[1, 1, 0, 2]) / np.float32(255) - np.float32(0.3)) / np.float32(0.5))
