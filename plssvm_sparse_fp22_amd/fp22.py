"""Packed FP22 host codec (numpy), the layout of PLSSVM_MI_VAL_FP22 (include/plssvm_mi355x.h).

FP22 = binary32 truncated to its top 22 bits (1 sign, 8 exponent, 13 mantissa) with
round-to-nearest-even on the 10 dropped bits; NaN stays NaN, +-Inf stay Inf. 16 values are
packed into 11 little-endian uint32 words, value k of a group at bits [22k, 22k+22).
Build-defined: the reference has no FP22.
"""
from __future__ import annotations

import numpy as np


def encode(v):
    u = np.ascontiguousarray(v, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x007FFFFF) != 0)
    code = ((u + 0x1FF + ((u >> 10) & 1)) >> 10) & 0x3FFFFF
    code = np.where(nan, ((u >> 10) | 0x1000) & 0x3FFFFF, code)
    return code.astype(np.uint32)


def decode(code):
    return (np.asarray(code, dtype=np.uint32) << np.uint32(10)).view(np.float32)


def n_words(n):
    return ((n + 15) // 16) * 11


def pack(v):
    code = encode(v)
    n = code.size
    g = (n + 15) // 16
    c = np.zeros(g * 16, dtype=np.uint64)
    c[:n] = code
    c = c.reshape(g, 16)
    words = np.zeros((g, 11), dtype=np.uint64)
    for k in range(16):
        bit = 22 * k
        w, s = bit // 32, bit % 32
        words[:, w] |= (c[:, k] << np.uint64(s)) & np.uint64(0xFFFFFFFF)
        if s + 22 > 32:
            words[:, w + 1] |= c[:, k] >> np.uint64(32 - s)
    return words.astype(np.uint32).reshape(-1)


def unpack(words, n):
    g = (n + 15) // 16
    w = np.asarray(words, dtype=np.uint64)[: g * 11].reshape(g, 11)
    out = np.zeros((g, 16), dtype=np.uint32)
    for k in range(16):
        bit = 22 * k
        i, s = bit // 32, bit % 32
        x = w[:, i] >> np.uint64(s)
        if s + 22 > 32:
            x |= w[:, i + 1] << np.uint64(32 - s)
        out[:, k] = (x & np.uint64(0x3FFFFF)).astype(np.uint32)
    return decode(out.reshape(-1)[:n])
