"""Radler::Perform's major-iteration state machine (cpp/radler.cc:130-316)
driven over the oracle's algorithms, for one single-channel image on a 1x1
grid or a subimage grid (oracle/tiling.cc): auto-threshold and auto-masking thresholds, the doubled gain once the
auto-mask is complete, the per-scale mask mode (multiscale) or the model's
non-zero mask (other algorithms), and the stopping rules.

TEST INFRASTRUCTURE: the checker for tests/test_automask.py (imports the
oracle); never used by the product.
"""
import numpy as np

from oracle_lib import OracleAlgorithm, OracleParallel


def median_and_stddev_from_mad(image):
    """aocommon Image::MedianAndStdDevFromMAD as the product computes it
    (rdl_median: exact median, mean of the two middle values for even n,
    in float): stddev = MAD * 1.48260221850560."""
    v = image.astype(np.float32).ravel()
    med = np.float32(np.median(v))
    mad = np.float32(np.median(np.abs(v - med)))
    return float(med), float(mad) * 1.48260221850560


class OraclePerform:
    def __init__(self, orc, kind, psf, dirty, *, minor_loop_gain=0.1, major_loop_gain=1.0,
                 absolute_threshold=0.0, auto_mask_sigma=None, auto_threshold_sigma=None,
                 absolute_auto_mask_threshold=None, minor_iteration_count=1000,
                 major_iteration_count=20, major_auto_mask_iteration_count=2,
                 grid=None, snapshot=False, local_rms=None, component_optimization=0,
                 **algo_settings):
        self.orc, self.kind = orc, kind
        self.psf = psf[None].astype(np.float32)
        self.residual = dirty[None].astype(np.float32).copy()
        self.model = np.zeros_like(self.residual)
        self.gain, self.mgain = minor_loop_gain, major_loop_gain
        self.abs_thr = absolute_threshold
        self.am_sigma, self.at_sigma = auto_mask_sigma, auto_threshold_sigma
        self.abs_am = absolute_auto_mask_threshold
        self.minor_count = minor_iteration_count
        self.major_count = major_iteration_count
        self.major_am_count = major_auto_mask_iteration_count
        self.algo_settings = algo_settings
        self.threshold = absolute_threshold
        self.finished = False
        self.finishing_iteration = 0
        self.auto_mask = None
        self.grid = grid
        # local_rms: None or dict(method=1|2, window, strength, beam, pixel_scale)
        self.local_rms = local_rms
        self.component_optimization = component_optimization  # 2: gradient descent
        if grid is None:
            self.alg = OracleAlgorithm(orc, kind, **self._settings(self.gain, None))
        else:  # ParallelDeconvolution::ExecuteParallelRun (oracle/tiling.cc)
            self.alg = OracleParallel(orc, kind, grid[0], grid[1],
                                      **self._settings(self.gain, None))
            self.alg.set_snapshot(snapshot)
        self.traces = []

    def _settings(self, gain, mask):
        st = dict(self.algo_settings)
        st.update(threshold=self.threshold, minor_loop_gain=gain,
                  major_loop_gain=self.mgain, max_iterations=self.minor_count)
        if mask is not None:
            st["clean_mask"] = mask
        return st

    def perform(self, major):
        """One Perform(major): returns another_iteration_required."""
        enabled = self.am_sigma is not None or self.abs_am is not None
        gain = min(1.0, self.gain * 2.0) if (enabled and self.finished) else self.gain
        if self.at_sigma is not None or enabled or self.local_rms:
            med, stddev = median_and_stddev_from_mad(self.residual[0])
            bias = 0.0
            if enabled and self.finished:  # cpp/radler.cc:172-185
                if self.local_rms:
                    self.alg.set_rms(None)
                if self.component_optimization:
                    self.alg.set_component_optimization(self.component_optimization)
            elif self.local_rms:  # cpp/radler.cc:196-216
                lr = self.local_rms
                _, factor, stddev = self.orc.local_rms(
                    self.residual[0], lr["method"], lr["window"], lr["beam"],
                    lr["pixel_scale"], lr["pixel_scale"], lr.get("strength", 1.0))
                self.alg.set_rms(factor)
                self.last_rms_factor = factor
            if enabled and not self.finished:
                am = max(stddev * (self.am_sigma or 0.0) + bias, self.abs_am or 0.0)
                self.threshold = max(am, self.abs_thr)
            elif self.at_sigma is not None:
                self.threshold = max(stddev * self.at_sigma + bias, self.abs_thr)
        mask = None
        if self.kind == 1:
            if enabled:
                self.alg.set_automask(not self.finished, self.finished)
        elif enabled and self.finished:
            if self.auto_mask is None:
                m = self.model[0]
                self.auto_mask = (np.isfinite(m) & (m != 0.0)).astype(np.uint8)
            mask = self.auto_mask
        if self.grid is None:
            self.alg.update(**self._settings(gain, mask))
            r, trace = self.alg.execute(self.residual, self.model, self.psf)
            self.iteration_number = r.iteration_number
        else:  # the mask goes to the subimage split (MakeSubImages' user mask)
            self.alg.update(**self._settings(gain, None))
            r, _, _, trace = self.alg.execute(self.residual, self.model, self.psf,
                                              self.mgain, user_mask=mask)
            self.iteration_number = r.first_iteration_number  # cpp/radler.cc:406-408
            self.total_iterations = r.total_iterations
        self.traces.append(trace)
        another = bool(r.another_iteration_required)
        if not another and enabled and not self.finished:
            self.finished, another = True, True
            self.finishing_iteration = major
        if another and self.major_count and major >= self.major_count:
            another = False
        if another and self.finished and major - self.finishing_iteration >= self.major_am_count:
            another = False
        if another and self.minor_count and self.iteration_number >= self.minor_count:
            another = False
        return another
