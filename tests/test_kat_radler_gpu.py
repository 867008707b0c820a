"""The reference's Radler-level known-answer tests that exercise the tiling
and direction-dependent PSFs, restated through the product's `radler`
module (Radler.perform on the MI355X):

* cpp/test/test_divergence.cc:26-142 — a 5 x 5 subimage grid with 25
  direction-dependent PSFs, one of which (subimage 19) has no central peak:
  that subimage diverges and is reset, every other one cleans its two
  sources, and the component list holds 2 x 25 - 2 = 48 components.
* python/test/test_psf.py:87-225 — a 3 x 3 grid of nine differently shaped
  PSFs; one Högbom iteration per subimage subtracts the PSF nearest to each
  source.
"""
import numpy as np
import pytest


def divergence_kat_failures():
    """Run the KAT through Radler.perform; every violated check as
    (box index, x, y, value, check) (an empty list: the KAT holds)."""
    from radler_import import radler as rd
    grid, sub = 5, 32
    width = height = sub * grid
    pixel_scale = 1.0 / 60.0 / 60.0 * (np.pi / 180.0)
    s = rd.Settings()
    s.trimmed_image_width, s.trimmed_image_height = width, height
    s.pixel_scale.x = s.pixel_scale.y = pixel_scale
    s.minor_iteration_count = 1000000
    s.absolute_threshold = 1.0e-6
    s.parallel.grid_width = s.parallel.grid_height = grid
    s.divergence_limit = 4.0
    s.algorithm_type = rd.AlgorithmType.generic_clean
    s.save_source_list = True

    center = (height // 2) * width + width // 2
    good = np.zeros((height, width), np.float32)
    good.flat[center] = 1.0
    bad = np.zeros((height, width), np.float32)
    bad.flat[center - 2] = 2.0
    bad.flat[center + 2] = 2.0
    residual = np.zeros((height, width), np.float32)
    offsets = []
    for y in range(grid):
        for x in range(grid):
            ix, iy = x * sub + sub // 2, y * sub + sub // 2
            offsets.append((ix, iy))
            residual[iy, ix] = 5.0
            residual[iy, ix + 2] = 3.0
    model = np.zeros_like(residual)
    table = rd.WorkTable(np.array(offsets, np.uint64), 1, 1)
    e = rd.WorkTableEntry()
    e.polarization = rd.Polarization.stokes_i
    e.image_weight = 1.0
    for i in range(25):  # subimage 19 (grid indices [3, 4]) diverges
        e.psfs.append(bad if i == 19 else good)
    e.residual = residual
    e.model = model
    table.add_entry(e)
    radler = rd.Radler(s, table, pixel_scale)
    radler.perform(1)

    fails = []

    def check(ok, i, bx, by, values, what):
        # the first violating pixel of the box (row-major), with its value
        ok = np.asarray(ok)
        if ok.all():
            return
        k = int(np.argmax(~ok.ravel()))
        y, x = divmod(k, ok.shape[-1]) if ok.ndim == 2 else (0, k)
        fails.append((i, bx + x, by + y, float(np.asarray(values).ravel()[k]), what))

    for y in range(grid):
        for x in range(grid):
            i = y * grid + x
            bx, by = x * sub, y * sub
            ix, iy = bx + sub // 2, by + sub // 2
            if i == 19:
                check(abs(model[iy, ix]) <= 1e-5, i, ix, iy, model[iy, ix], "model source")
                check(abs(model[iy, ix + 2]) <= 1e-5, i, ix + 2, iy, model[iy, ix + 2],
                      "model source")
            else:
                check(abs(model[iy, ix] - 5.0) <= 5e-3, i, ix, iy, model[iy, ix], "model 5")
                check(abs(model[iy, ix + 2] - 3.0) <= 3e-3, i, ix + 2, iy, model[iy, ix + 2],
                      "model 3")
            r = residual[by:by + sub, bx:bx + sub]
            m = model[by:by + sub, bx:bx + sub]
            check(np.isfinite(r) & np.isfinite(m), i, bx, by, r, "finite")
            source = np.zeros((sub, sub), bool)
            source[sub // 2, sub // 2] = source[sub // 2, sub // 2 + 2] = True
            check_r = ~source if i == 19 else np.ones_like(source)
            check(~check_r | (r < 1e-5), i, bx, by, r, "residual < 1e-5")
            check_m = np.ones_like(source) if i == 19 else ~source
            check(~check_m | (np.abs(m) < 1e-5), i, bx, by, m, "|model| < 1e-5")
    n = radler.component_list.component_count(0)
    if n != grid * grid * 2 - 2:
        fails.append((-1, 0, 0, float(n), "component count 48"))
    return fails


@pytest.mark.gpu
def test_divergence_kat():
    fails = divergence_kat_failures()
    assert not fails, f"violated checks (box, x, y, value, check): {fails[:10]}"


def psf_rectangular(size, w, h):
    psf = np.zeros((size, size), np.float32)
    psf[size // 2 - h:size // 2 + h + 1, size // 2 - w:size // 2 + w + 1] = 0.4
    psf[size // 2, size // 2] = 1
    return psf


def psf_cross(size, w, h):
    psf = np.zeros((size, size), np.float32)
    psf[size // 2 - h:size // 2 + h + 1, size // 2] = 0.4
    psf[size // 2, size // 2 - w:size // 2 + w + 1] = 0.4
    psf[size // 2, size // 2] = 1
    return psf


def subimage(cx, cy, interval, img):
    return img[cx - interval:cx + interval + 1, cy - interval:cy + interval + 1]


def check_values(psf, residual, psf_center, source):
    r = subimage(psf_center[0], psf_center[1], 15, residual)
    r = subimage(source[0] % 30, source[1] % 30, 5, r)
    p = subimage(psf.shape[0] // 2, psf.shape[1] // 2, 5, psf)
    combined = r + p
    np.testing.assert_allclose(combined[combined.shape[0] // 2, combined.shape[0] // 2], 1,
                               rtol=1e-5, atol=1e-6)
    combined[5, 5] = 0
    np.testing.assert_allclose(combined, np.zeros_like(combined), rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_direction_dependent_psfs_kat():
    from radler_import import radler as rd
    image_size = 90
    psf_size = image_size // 3
    center_offset = psf_size // 2
    psf_centers = np.zeros((9, 2), dtype=np.int64)
    for i in range(3):
        for k in range(3):
            psf_centers[3 * i + k] = [i * image_size // 3 + center_offset,
                                      k * image_size // 3 + center_offset]
    work_table = rd.WorkTable(psf_centers, 0, 0)
    w1, w2, w3 = 2, 4, 8
    psfs = [psf_rectangular(psf_size, w2, w2), psf_cross(psf_size, w2, w2),
            psf_cross(psf_size, w1, w3), psf_rectangular(psf_size, w2, 0),
            psf_cross(psf_size, w3, w1), psf_rectangular(psf_size, w2, w1),
            psf_rectangular(psf_size, 0, w2), psf_rectangular(psf_size, 0, 0),
            psf_rectangular(psf_size, w1, w2)]
    residual = np.zeros((image_size, image_size), np.float32)
    rng = np.random.RandomState(10)  # np.random.seed(10) + randint in the reference
    source_coords = np.zeros((9, 2), dtype=np.int64)
    for i in range(3):
        for k in range(3):
            off = rng.randint(-4, 4)
            source_coords[3 * i + k] = psf_centers[3 * i + k] + off
    for p in source_coords:
        residual[p[0], p[1]] = 1
    model = np.zeros((image_size, image_size), np.float32)
    entry = rd.WorkTableEntry()
    for psf in psfs:
        entry.psfs.append(psf)
    entry.residual = residual
    entry.model = model
    entry.polarization = rd.Polarization.stokes_i
    entry.image_weight = 1.0
    work_table.add_entry(entry)
    s = rd.Settings()
    s.algorithm_type = rd.AlgorithmType.generic_clean
    s.trimmed_image_width = s.trimmed_image_height = image_size
    s.pixel_scale.x = s.pixel_scale.y = 1.0
    s.minor_iteration_count = 1
    s.minor_loop_gain = 1.0
    s.parallel.grid_width = s.parallel.grid_height = 3
    s.parallel.max_threads = 1
    radler = rd.Radler(s, work_table, 0)
    radler.perform(0)
    # the PSF nearest to each source (test_psf.py:199-225)
    for psf_index, cell in [(0, 0), (3, 1), (6, 2), (1, 3), (4, 4), (7, 5), (2, 6), (5, 7),
                            (8, 8)]:
        check_values(psfs[psf_index], residual, psf_centers[cell], source_coords[cell])
