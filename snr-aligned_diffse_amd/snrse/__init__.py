"""snrse — MI355X-native runtime of the SNR-aligned diffusion speech-enhancement path.

Host side (PyTorch-ROCm for device memory / streams) over libsnrse_hip.so (HIP kernels
for gfx950, C-ABI in include/snrse.h).  The reference-compatible module API lives in the
sibling `sgmse` package.
"""
__all__ = ["ops", "ncsnpp", "sampler", "formula"]
