"""Drop-in `sgmse` package backed by the MI355X-native snrse runtime.

Same module paths, class names and call signatures as the reference's sgmse-bbed/sgmse
(model, sdes, sampling, backbones, data_module, snr_estimator, util) for the inference
path ScoreModel.enhance() / PC sampler, so eval.py / deep_eval.py run unchanged.  Compute
goes through libsnrse_hip.so (HIP kernels for gfx950); there is no CPU fallback.
"""
import os as _os
import sys as _sys

_pkg_root = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _pkg_root not in _sys.path:
    _sys.path.insert(0, _pkg_root)
