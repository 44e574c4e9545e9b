"""MX-FP8 (OCP e4m3fn elements, E8M0 scale per 32-element block) quantisation — ORACLE (test
infra only).

Config 5 of SURVEY §8(d) runs the decoder output-layer and regulariser GEMMs (model.py:64,94,98)
on the gfx950 block-scaled MFMA (v_mfma_scale_f32_32x32x64_f8f6f4).  The reference has no fp8
path (TF fp32, train.py:83-88); parity there is claimed at fp32 only (§8(d) "Config 5"), so this
module pins only the build's own quantiser, bit for bit, and the GEMM on dequantised operands.

Rule (both here and in csrc/gemm.hip quant kernels):
  * a block is 32 consecutive elements along the GEMM's K axis (zero padding past the end);
  * scale exponent e = the smallest integer with amax <= 448 * 2^e (448 = largest e4m3 normal),
    i.e. with amax = m 2^x (m in [0.5, 1)): e = x - 9 + (m > 0.875); all-zero block: e = 0;
    e clamped to [-127, 127], E8M0 byte = e + 127;
  * element code = e4m3fn round-to-nearest-even of x * 2^-e (never saturates by construction);
    the sign bit is kept when the magnitude rounds to zero (-0 = 0x80), as v_cvt_pk_fp8_f32 does.
"""
import numpy as np

_POS = np.array([((1 + (c & 7) / 8.0) * 2.0 ** ((c >> 3) - 7)) if (c >> 3) else (c & 7) / 8.0 * 2.0 ** -6
                 for c in range(0x7F)], np.float64)   # codes 0x00..0x7E (0x7F is NaN)


def e4m3_decode(codes):
    c = np.asarray(codes, np.uint8)
    mag = _POS[np.minimum(c & 0x7F, 0x7E)]
    return np.where(c & 0x80, -mag, mag)


def e4m3_encode(x):
    """Round-to-nearest-even e4m3fn codes of |x| <= 448 (float array)."""
    x = np.asarray(x, np.float64)
    a = np.abs(x)
    hi = np.clip(np.searchsorted(_POS, a, side='left'), 0, 0x7E)
    lo = np.maximum(hi - 1, 0)
    dlo, dhi = a - _POS[lo], _POS[hi] - a
    pick_hi = (dhi < dlo) | ((dhi == dlo) & ((hi & 1) == 0))
    code = np.where(pick_hi, hi, lo).astype(np.uint8)
    code = np.where(a == _POS[hi], hi, code).astype(np.uint8)
    return np.where(np.signbit(x), code | 0x80, code).astype(np.uint8)   # sign kept, also on zero


def block_exponent(amax):
    amax = np.asarray(amax, np.float32)
    m, x = np.frexp(amax)
    e = x.astype(np.int64) - 9 + (m > 0.875)
    return np.clip(np.where(amax > 0, e, 0), -127, 127)


def quantize_rows(X, K_pad=None):
    """X [rows, K] (fp32/bf16-valued) -> (codes [rows, K_pad] u8, scales [rows, K_pad/32] u8)."""
    X = np.asarray(X, np.float32)
    rows, K = X.shape
    Kp = K_pad or -(-K // 32) * 32
    Xp = np.zeros((rows, Kp), np.float32)
    Xp[:, :K] = X
    blk = Xp.reshape(rows, Kp // 32, 32)
    e = block_exponent(np.abs(blk).max(2))
    codes = e4m3_encode(blk.astype(np.float64) * np.exp2(-e)[..., None].astype(np.float64))
    return codes.reshape(rows, Kp), (e + 127).astype(np.uint8)


def dequantize_rows(codes, scales):
    rows, Kp = codes.shape
    v = e4m3_decode(codes).reshape(rows, Kp // 32, 32)
    return (v * np.exp2(scales.astype(np.float64) - 127)[..., None]).reshape(rows, Kp)
