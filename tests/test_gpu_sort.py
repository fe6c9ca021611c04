"""GPU parity of the radix sort (gs_argsort_f32 / gs_sort_pairs_u32) -- mirrors the
reference's SortTest.SortTest (tests/sortTests.cpp:127-253), then edge sizes and key
distributions.  Bar: bit-exact stable permutation."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SORT_N = 32 * 16 * 10000 - 7
GOLD_FNV_SORTED_KEYS = 0xF7C786D96C9BBF6A
GOLD_FNV_PERMUTATION = 0x127693EABFDBBEA9


@pytest.fixture(scope="module")
def ctx():
    import openglgaussiansplattingrenderer_amd as g
    c = g.Context(0)
    yield c
    c.close()


def gpu_argsort(ctx, keys, order=None):
    import openglgaussiansplattingrenderer_amd as g
    keys = np.ascontiguousarray(keys, np.float32)
    n = len(keys)
    order = np.arange(n, dtype=np.int32) if order is None else np.ascontiguousarray(order, np.int32)
    kb = g.DeviceBuffer.from_array(ctx, keys if n else np.zeros(1, np.float32))
    ob = g.DeviceBuffer.from_array(ctx, order if n else np.zeros(1, np.int32))
    g.GPURadixSort(1, 3, 2, None, ob, None, n, 16, 32, kb)
    return ob.download(np.int32, n)


def test_sort_test_mirror(ctx, oracle):
    """tests/sortTests.cpp:181-244: 5,119,993 srand(20) keys, GPURadixSort(..., size, 16, 32)"""
    import openglgaussiansplattingrenderer_amd as g
    g.createAndLinkSortAndHistogramShaders()
    keys = oracle.gen_sort_keys(SORT_N)
    out = gpu_argsort(ctx, keys)
    s = keys[out]
    assert np.all(s[1:] >= s[:-1])                        # sortTests.cpp:241
    assert np.array_equal(s, np.sort(keys))               # sortTests.cpp:242
    assert oracle.fnv1a64_words(keys.view(np.uint32)[out]) == GOLD_FNV_SORTED_KEYS
    assert oracle.fnv1a64_words(out) == GOLD_FNV_PERMUTATION
    assert np.array_equal(out, oracle.argsort_f32(keys))


@pytest.mark.parametrize("n", [0, 1, 2, 3, 63, 64, 65, 1000, 4095, 4096, 4097, 8191, 10_000, 20_000, 100_003,
                               262_143, 1_000_003])
def test_argsort_sizes(ctx, n):
    rng = np.random.default_rng(n)
    keys = (rng.integers(0, 300, n) + rng.integers(0, 3, n) * 0.5).astype(np.float32)
    keys[rng.random(n) < 0.1] *= -1  # negatives sort after positives by bits
    out = gpu_argsort(ctx, keys)
    assert np.array_equal(out, np.argsort(keys.view(np.uint32), kind="stable"))


def test_argsort_respects_initial_order(ctx):
    """order is read as the initial sequence (scan.glsl:337): stable w.r.t. it"""
    rng = np.random.default_rng(11)
    n = 70_001
    keys = rng.integers(0, 50, n).astype(np.float32)
    order = rng.permutation(n).astype(np.int32)
    out = gpu_argsort(ctx, keys, order)
    exp = order[np.argsort(keys[order].view(np.uint32), kind="stable")]
    assert np.array_equal(out, exp)


@pytest.mark.parametrize("dist", ["uniform32", "equal", "top_byte_const", "descending", "two_values", "render_like"])
def test_sort_pairs_distributions(ctx, dist):
    import openglgaussiansplattingrenderer_amd as g
    rng = np.random.default_rng(5)
    n = 1_234_567
    if dist == "uniform32":
        k = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    elif dist == "equal":
        k = np.full(n, 0xDEADBEEF, np.uint32)
    elif dist == "top_byte_const":
        k = (0x42000000 | rng.integers(0, 2**24, n)).astype(np.uint32)
    elif dist == "descending":
        k = np.arange(n, 0, -1).astype(np.uint32)
    elif dist == "two_values":
        k = np.where(rng.random(n) < 0.5, 7, 0x80000000).astype(np.uint32)
    else:  # tile + z01 float keys
        k = (rng.integers(0, 256, n) + rng.random(n) * 0.02 + 0.97).astype(np.float32).view(np.uint32)
    v = np.arange(n, dtype=np.uint32) * 3
    kb, vb = g.DeviceBuffer.from_array(ctx, k), g.DeviceBuffer.from_array(ctx, v)
    g.sort_pairs(ctx, kb, vb, n)
    ks, vs = kb.download(np.uint32, n), vb.download(np.uint32, n)
    o = np.argsort(k, kind="stable")
    assert np.array_equal(ks, k[o])
    assert np.array_equal(vs, v[o])


@pytest.mark.parametrize("dist", ["uniform32", "top_byte_const"])
def test_sort_pairs_beyond_16M(ctx, dist):
    """standalone pair sorts of >= 16M keys take the 8-wave form in every pass, with the upsweeps
    walking each XCD's tile range backwards (k_upsweep REV): a ragged size past 2^24, bit-exact
    stable pairs"""
    import openglgaussiansplattingrenderer_amd as g
    rng = np.random.default_rng(24)
    n = (1 << 24) + 12_345
    if dist == "uniform32":
        k = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    else:
        k = (0x42000000 | rng.integers(0, 2**24, n)).astype(np.uint32)
    v = np.arange(n, dtype=np.uint32)
    kb, vb = g.DeviceBuffer.from_array(ctx, k), g.DeviceBuffer.from_array(ctx, v)
    g.sort_pairs(ctx, kb, vb, n)
    ks, vs = kb.download(np.uint32, n), vb.download(np.uint32, n)
    o = np.argsort(k, kind="stable")
    assert np.array_equal(ks, k[o])
    assert np.array_equal(vs, o.astype(np.uint32))
