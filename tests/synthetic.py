"""Deterministic synthetic skies for parity tests and the benchmark
(SURVEY.md §8(d) "Synthetic inputs", scaled down for the parity sizes)."""
import numpy as np


def make_psf(w, h, fwhm=4.0, pa_deg=30.0, axis_ratio=0.7, sidelobe=0.05):
    """Analytic dirty beam: elliptical Gaussian core + ring sidelobes,
    psf[h//2, w//2] == 1.0 exactly."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    dx, dy = xx - w // 2, yy - h // 2
    pa = np.deg2rad(pa_deg)
    u = dx * np.cos(pa) + dy * np.sin(pa)
    v = -dx * np.sin(pa) + dy * np.cos(pa)
    s = fwhm / 2.3548
    core = np.exp(-0.5 * ((u / s) ** 2 + (v / (s * axis_ratio)) ** 2))
    r = np.hypot(dx, dy)
    psf = core + sidelobe * np.cos(2 * np.pi * r / 9.0) * np.exp(-r / 40.0)
    psf /= psf[h // 2, w // 2]
    out = psf.astype(np.float32)
    out[h // 2, w // 2] = 1.0
    return out


def make_psf_uv(w, h, fwhm=4.0, pa_deg=30.0, axis_ratio=0.7, ring_px=9.0, ring_depth=0.4):
    """Dirty beam synthesised from a non-negative uv weighting, as an
    interferometer's is: W(u,v) = elliptical Gaussian taper (the FWHM-`fwhm`
    core) x (1 - ring_depth/2 + ring_depth/2 cos(2 pi ring_px |uv|)) >= 0, whose
    inverse FFT gives ring sidelobes at ~ring_px with a peak at the centre.
    A non-negative spectrum keeps CLEAN convergent (make_psf's ring sidelobes
    have a negative spectrum and make long CLEAN runs diverge).
    psf[h//2, w//2] == 1.0 exactly."""
    u = np.fft.fftfreq(w)[None, :]
    v = np.fft.fftfreq(h)[:, None]
    pa = np.deg2rad(pa_deg)
    # image-plane sigma along the two axes -> uv-plane sigma 1/(2 pi sigma)
    sx = fwhm / 2.3548
    sy = sx * axis_ratio
    uu = u * np.cos(pa) + v * np.sin(pa)
    vv = -u * np.sin(pa) + v * np.cos(pa)
    taper = np.exp(-2.0 * np.pi ** 2 * ((uu * sx) ** 2 + (vv * sy) ** 2))
    r = np.hypot(u, v)
    cover = 1.0 - ring_depth / 2 + ring_depth / 2 * np.cos(2.0 * np.pi * ring_px * r)
    psf = np.fft.fftshift(np.fft.ifft2(taper * cover).real)
    psf /= psf[h // 2, w // 2]
    out = psf.astype(np.float32)
    out[h // 2, w // 2] = 1.0
    return out


def make_sky(w, h, n_points, n_blobs, seed, margin=16, flux_range=(1e-3, 1.0),
             blob_sigma=(2.0, 40.0)):
    rng = np.random.default_rng(seed)
    sky = np.zeros((h, w), np.float64)
    xs = rng.integers(margin, w - margin, n_points)
    ys = rng.integers(margin, h - margin, n_points)
    fl = np.exp(rng.uniform(np.log(flux_range[0]), np.log(flux_range[1]), n_points))
    np.add.at(sky, (ys, xs), fl)
    if n_blobs:
        yy, xx = np.ogrid[0:h, 0:w]  # broadcast views: same values as mgrid
        for _ in range(n_blobs):
            cx, cy = rng.uniform(margin, w - margin), rng.uniform(margin, h - margin)
            sg = np.exp(rng.uniform(np.log(blob_sigma[0]), np.log(blob_sigma[1])))
            amp = np.exp(rng.uniform(np.log(flux_range[0]), np.log(flux_range[1]))) / (sg * sg)
            x0, x1 = int(max(0, cx - 5 * sg)), int(min(w, cx + 5 * sg + 1))
            y0, y1 = int(max(0, cy - 5 * sg)), int(min(h, cy + 5 * sg + 1))
            sky[y0:y1, x0:x1] += amp * np.exp(
                -0.5 * ((xx[:, x0:x1] - cx) ** 2 + (yy[y0:y1, :] - cy) ** 2) / (sg * sg))
    return sky


def make_dirty(psf, sky, noise, seed):
    """dirty = sky (*) psf (circular, float64 FFT) + Gaussian noise."""
    h, w = sky.shape
    rng = np.random.default_rng(seed + 1)
    P = np.fft.rfft2(np.fft.ifftshift(psf.astype(np.float64)))
    dirty = np.fft.irfft2(np.fft.rfft2(sky) * P, s=(h, w))
    dirty += noise * rng.standard_normal((h, w))
    return dirty.astype(np.float32)


def problem(w, h, n_points=40, n_blobs=4, seed=2025, noise=1e-3, fwhm=4.0):
    psf = make_psf(w, h, fwhm=fwhm)
    sky = make_sky(w, h, n_points, n_blobs, seed)
    return psf, make_dirty(psf, sky, noise, seed)
