"""The bucket sort's first digit (gs_sort.hip bucket_of): int(key) as a float below 255.0's bits,
255 from them on.  A stable scatter by it followed by a stable per-bucket sort is the stable sort
of the keys only if it is monotone in the unsigned key -- checked here over every kind of bit
pattern a frame's keys can hold (tile + depth floats, depths outside [0, 1] in ref mode, the
culled 1e6, +inf, NaN, negative floats)."""
import numpy as np

BITS_255 = 0x437F0000


def bucket_of(keys: np.ndarray) -> np.ndarray:
    k = keys.astype(np.uint32)
    f = k.view(np.float32)
    with np.errstate(invalid="ignore"):
        t = np.trunc(np.where(np.isnan(f), 0.0, f)).astype(np.int64)  # v_cvt_i32_f32 (below 255: in range)
    return np.where(k >= BITS_255, 255, t)


def test_bucket_of_is_monotone_in_the_key_bits():
    rng = np.random.default_rng(0)
    tiles = rng.integers(0, 256, 200_000).astype(np.float32)
    z = rng.uniform(-1.5, 2.5, 200_000).astype(np.float32)
    keys = np.concatenate([
        (tiles + z).view(np.uint32),                                          # frame keys, ref-mode depths
        rng.integers(0, 2**32, 200_000, dtype=np.uint64).astype(np.uint32),   # any bit pattern
        np.array([0, 1, BITS_255 - 1, BITS_255, 0x3F800000, 0x49742400,       # 1.0, 1e6
                  0x7F800000, 0x7FC00000, 0x80000000, 0xFF800000, 0xFFFFFFFF], np.uint32),
    ])
    s = np.sort(keys)
    b = bucket_of(s)
    assert b.min() >= 0 and b.max() <= 255
    assert np.all(np.diff(b) >= 0)
    # and each tile's keys [t, t + 1) land in bucket t
    ok = (z >= 0) & (z < 1) & ((tiles + z) < tiles + 1)
    assert np.array_equal(bucket_of((tiles + z).view(np.uint32))[ok], tiles[ok].astype(np.int64))


def bucket_form(keys: np.ndarray, vals: np.ndarray):
    """numpy restatement of the bucket form (gs_sort.hip k_sweep_small<BKT> + k_bucket_sort):
    stable scatter by bucket_of, then per bucket the 8-bit LSD passes over the bits below the
    highest one where its smallest and largest key differ (bucket_passes)"""
    b = bucket_of(keys)
    o = np.argsort(b, kind="stable")
    k, v, b = keys[o], vals[o], b[o]
    for d in np.unique(b):
        idx = np.nonzero(b == d)[0]
        kk, vv = k[idx], v[idx]
        diff = int(kk.min()) ^ int(kk.max())
        passes = (diff.bit_length() + 7) // 8
        for p in range(passes):
            oo = np.argsort((kk >> np.uint32(8 * p)) & np.uint32(0xFF), kind="stable")
            kk, vv = kk[oo], vv[oo]
        k[idx], v[idx] = kk, vv
    return k, v


def test_bucket_form_is_the_stable_sort_of_ref_mode_keys():
    """the withdrawn GPU scene's key kinds (NDC depths -1.5..2.5 in ref mode: keys below their
    tile, negative floats for tile 0, keys past tile + 1), the culled 1e6 entries and ties: the
    bucket form's order is the stable sort by the unsigned key bits"""
    rng = np.random.default_rng(7)
    n = 60_000
    tiles = rng.integers(0, 256, n).astype(np.float32)
    tiles[: n // 8] = 0.0  # tile 0: depths below 0 give negative floats (bucket 255)
    z = rng.uniform(-1.5, 2.5, n).astype(np.float32)
    keys = (tiles + z).view(np.uint32).copy()
    keys[rng.random(n) < 0.05] = 0x49742400  # culled entries: 1e6
    keys[rng.random(n) < 0.05] = keys[0]     # ties
    vals = np.arange(n, dtype=np.uint32)
    k, v = bucket_form(keys, vals)
    o = np.argsort(keys, kind="stable")
    assert np.array_equal(k, keys[o])
    assert np.array_equal(v, vals[o])
