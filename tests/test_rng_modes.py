"""Statistical pin of the build's per-path RNG against the reference's own
execution model.

Mode A (oracle_reference_compute) is the reference as written: ONE sequential
xorshift32 stream (rng.rs:11) shared by RandomSamplingStrategy's pixel picks
(sampling_strategy.rs:56-59) and every path, compute(n) splitting n/2 left
and n - n/2 right (wasm_interface.rs:374-379). Mode B (oracle render) is what
the GPU core computes: per-path streams path_seed(seed, pixel, sample), raster
pixel order, same draw order inside a path. The two cannot agree bit for bit;
they must estimate the same image. Each mode is run as R independent replicas
(different stream seeds); per 8x8 tile the replica means of the two modes are
compared with a Welch z-score, and the image-level L2 between the modes is
compared with the Monte-Carlo error predicted by the replica variances.
"""
import numpy as np
import pytest

W, H, TILE, R = 48, 48, 8, 10
SPP = 32          # mode B samples per pixel and replica; mode A takes the same budget at random pixels
DEPTH = 0         # the reference's unbounded Russian-roulette loop


def _tiles(img, cnt):
    t = img.reshape(H // TILE, TILE, W // TILE, TILE, 3).sum(axis=(1, 3))
    c = cnt.reshape(H // TILE, TILE, W // TILE, TILE).sum(axis=(1, 3))
    return (t / c[..., None]).reshape(-1, 3), c.reshape(-1)


def _replicas(wpt, oracle, types_a, types_b):
    cloud = wpt.scenes.triangle_cloud(1500, seed=0xC10D)
    sc = oracle.OracleScene(2, cloud)
    cam = wpt.scenes.scene_camera(2)
    types = types_a
    a_means, b_means, a_imgs, b_imgs = [], [], [], []
    for r in range(R):
        acc_b, _ = sc.render(W, H, cam, types_b[0], types_b[1], DEPTH, 0x1234567 + 7919 * r, 0, SPP, threads=8)
        cnt_b = np.full((H, W), SPP, np.uint32)
        acc_a, cnt_a, _, _ = sc.reference_compute(W, H, cam, W * H * SPP, types[0], types[1], DEPTH,
                                                  rng_state=(0xBABABEBE + 104729 * r) & 0xFFFFFFFF)
        assert int(cnt_a.sum()) == W * H * SPP
        assert int(cnt_a[:, : W // 2].sum()) == (W * H * SPP) // 2  # the reference's half split
        b_means.append(_tiles(acc_b, cnt_b)[0])
        a_means.append(_tiles(acc_a, cnt_a)[0])
        b_imgs.append(acc_b / SPP)
        a_imgs.append(acc_a / np.maximum(cnt_a, 1)[..., None])
    return np.array(a_means), np.array(b_means), np.array(a_imgs), np.array(b_imgs)


@pytest.fixture(scope="module")
def replicas(wpt, oracle):
    return _replicas(wpt, oracle, (0, 1), (0, 1))  # NoNEE left, NormalNEE right, in both modes


def _tile_z(a, b):
    ma, mb = a.mean(0), b.mean(0)
    va, vb = a.var(0, ddof=1) / R, b.var(0, ddof=1) / R
    lit = (ma + mb) > 1e-3                    # tiles that receive light at all
    return (ma - mb)[lit] / np.sqrt(va + vb + 1e-12)[lit]


def test_tile_means_agree(replicas):
    a, b, _, _ = replicas                     # (R, tiles, 3)
    z = _tile_z(a, b)
    print(f"tiles {len(z)}, mean z^2 {np.mean(z ** 2):.3f}, max |z| {np.abs(z).max():.2f}")
    assert len(z) > 80  # lit (tile, channel) pairs of the 36 tiles
    # under H0 z is ~ t with 2R-2 dof: E[z^2] ~ 1.2; a bias of a few per cent per tile would blow it up
    assert np.mean(z ** 2) < 2.5
    assert np.mean(np.abs(z) > 4.0) < 0.01


def test_image_l2_within_monte_carlo_error(replicas):
    _, _, ia, ib = replicas                   # (R, H, W, 3) per-replica pixel means
    ma, mb = ia.mean(0), ib.mean(0)
    # expected squared distance of two independent unbiased estimates
    expect = (ia.var(0, ddof=1) / R + ib.var(0, ddof=1) / R).sum()
    got = ((ma - mb) ** 2).sum()
    rel = np.sqrt(got) / np.linalg.norm(mb)
    print(f"|A-B|^2 {got:.4g} vs Monte-Carlo expectation {expect:.4g} (rel L2 {rel:.3e})")
    assert 0.5 * expect < got < 1.6 * expect


def test_power_against_a_real_difference(wpt, oracle):
    """Negative control: the same comparison with NormalNEE instead of NoNEE
    on mode B's left half (the reference's NEE adds about half the direct
    light NoNEE does) must be rejected, so the tests above
    have the power to see a bias of that kind."""
    a, b, _, _ = _replicas(wpt, oracle, (0, 1), (1, 1))
    z = _tile_z(a, b)
    print(f"control: mean z^2 {np.mean(z ** 2):.1f}")
    assert np.mean(z ** 2) > 10.0
