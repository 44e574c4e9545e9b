"""MI355X-native hot path of the CubeCobra denoising-autoencoder recommender.

Host side (this package, PyTorch-ROCm for memory/streams/RCCL) over a C-ABI HIP library
(libccrec_hip.so, include/ccrec.h).  See DESIGN.md.
"""
__version__ = '0.1.0'
