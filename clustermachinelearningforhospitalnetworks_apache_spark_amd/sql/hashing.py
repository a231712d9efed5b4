"""Spark's row hash functions: ``hash`` (Murmur3 x86_32, seed 42) and ``xxhash64`` (XXH64, seed 42),
bit-exact with Spark's ``Murmur3Hash`` / ``XxHash64`` expressions.

Each column's value is hashed with the running hash of the previous columns as its seed (nulls
leave it unchanged). Numeric, boolean, date and timestamp columns are hashed on the device with
int64 tensor arithmetic (wrap-around multiplication, masked 32-bit lanes for Murmur3), so a column
of 100M rows is a handful of elementwise kernels; strings, arrays, structs and maps are hashed on
the host with the same integer recipes.

Type recipes (Spark): int-like / date / boolean → hashInt; long / timestamp → hashLong; float →
hashInt(floatToIntBits), double → hashLong(doubleToLongBits), with -0.0 as 0.0 and one NaN; strings
→ hashUnsafeBytes over UTF-8 (Murmur3's legacy per-byte tail); arrays / structs fold their elements.
"""
from __future__ import annotations

import struct as _struct
from typing import Any

import torch

from . import types as T

M32 = 0xFFFFFFFF
M64 = (1 << 64) - 1
_C1, _C2 = 0xCC9E2D51, 0x1B873593

P1 = 0x9E3779B185EBCA87
P2 = 0xC2B2AE3D27D4EB4F
P3 = 0x165667B19E3779F9
P4 = 0x85EBCA77C2B2AE63
P5 = 0x27D4EB2F165667C5


def _s64(c: int) -> int:
    c &= M64
    return c - (1 << 64) if c >= (1 << 63) else c


# ------------------------------------------------------------------------------------------ Murmur3 (host)

def _rotl32(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & M32


def _mixk1(k: int) -> int:
    k = (k * _C1) & M32
    k = _rotl32(k, 15)
    return (k * _C2) & M32


def _mixh1(h: int, k: int) -> int:
    h ^= k
    h = _rotl32(h, 13)
    return (h * 5 + 0xE6546B64) & M32


def _fmix32(h: int, n: int) -> int:
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    return h ^ (h >> 16)


def m3_int(v: int, seed: int) -> int:
    return _fmix32(_mixh1(seed & M32, _mixk1(v & M32)), 4)


def m3_long(v: int, seed: int) -> int:
    h = _mixh1(seed & M32, _mixk1(v & M32))
    h = _mixh1(h, _mixk1((v >> 32) & M32))
    return _fmix32(h, 8)


def m3_bytes(b: bytes, seed: int) -> int:
    n = len(b)
    aligned = n - n % 4
    h = seed & M32
    for i in range(0, aligned, 4):
        h = _mixh1(h, _mixk1(int.from_bytes(b[i:i + 4], "little")))
    for i in range(aligned, n):
        byte = b[i] - 256 if b[i] >= 128 else b[i]  # Java byte, sign-extended
        h = _mixh1(h, _mixk1(byte & M32))
    return _fmix32(h, n)


# ------------------------------------------------------------------------------------------ XXH64 (host)

def _rotl64(x: int, r: int) -> int:
    x &= M64
    return ((x << r) | (x >> (64 - r))) & M64


def _xx_fmix(h: int) -> int:
    h ^= h >> 33
    h = (h * P2) & M64
    h ^= h >> 29
    h = (h * P3) & M64
    return h ^ (h >> 32)


def xx_int(v: int, seed: int) -> int:
    h = (seed + P5 + 4) & M64
    h ^= ((v & M32) * P1) & M64
    h = (_rotl64(h, 23) * P2 + P3) & M64
    return _xx_fmix(h)


def xx_long(v: int, seed: int) -> int:
    h = (seed + P5 + 8) & M64
    h ^= (_rotl64((v & M64) * P2, 31) * P1) & M64
    h = (_rotl64(h, 27) * P1 + P4) & M64
    return _xx_fmix(h)


def _xx_round(acc: int, lane: int) -> int:
    acc = (acc + lane * P2) & M64
    return (_rotl64(acc, 31) * P1) & M64


def xx_bytes(b: bytes, seed: int) -> int:
    n = len(b)
    i = 0
    seed &= M64
    if n >= 32:
        v1 = (seed + P1 + P2) & M64
        v2 = (seed + P2) & M64
        v3 = seed
        v4 = (seed - P1) & M64
        while i <= n - 32:
            v1 = _xx_round(v1, int.from_bytes(b[i:i + 8], "little"))
            v2 = _xx_round(v2, int.from_bytes(b[i + 8:i + 16], "little"))
            v3 = _xx_round(v3, int.from_bytes(b[i + 16:i + 24], "little"))
            v4 = _xx_round(v4, int.from_bytes(b[i + 24:i + 32], "little"))
            i += 32
        h = (_rotl64(v1, 1) + _rotl64(v2, 7) + _rotl64(v3, 12) + _rotl64(v4, 18)) & M64
        for v in (v1, v2, v3, v4):
            h ^= _xx_round(0, v)
            h = (h * P1 + P4) & M64
    else:
        h = (seed + P5) & M64
    h = (h + n) & M64
    while i <= n - 8:
        h ^= _xx_round(0, int.from_bytes(b[i:i + 8], "little"))
        h = (_rotl64(h, 27) * P1 + P4) & M64
        i += 8
    if i <= n - 4:
        h ^= (int.from_bytes(b[i:i + 4], "little") * P1) & M64
        h = (_rotl64(h, 23) * P2 + P3) & M64
        i += 4
    while i < n:
        h ^= (b[i] * P5) & M64
        h = (_rotl64(h, 11) * P1) & M64
        i += 1
    return _xx_fmix(h)


# ------------------------------------------------------------------------------------------ values (host)

def _double_bits(v: float) -> int:
    if v != v:
        return 0x7FF8000000000000
    if v == 0.0:
        return 0
    return _struct.unpack("<q", _struct.pack("<d", v))[0]


def _float_bits(v: float) -> int:
    if v != v:
        return 0x7FC00000
    if v == 0.0:
        return 0
    return _struct.unpack("<i", _struct.pack("<f", v))[0]


def _unscaled(v: Any, scale: int) -> int:
    from decimal import ROUND_HALF_UP, Decimal
    d = v if isinstance(v, Decimal) else Decimal(repr(float(v)))
    return int(d.scaleb(scale).to_integral_value(rounding=ROUND_HALF_UP))


def hash_value(v: Any, dt: T.DataType, seed: int, algo: str) -> int:
    """Hash one Python value of Spark type ``dt`` (unsigned result in the algorithm's width)."""
    from .column import ts_to_micros
    fi, fl, fb = (m3_int, m3_long, m3_bytes) if algo == "murmur3" else (xx_int, xx_long, xx_bytes)
    if v is None:
        return seed
    if isinstance(dt, T.BooleanType):
        return fi(1 if v else 0, seed)
    if isinstance(dt, (T.ByteType, T.ShortType, T.IntegerType)):
        return fi(int(v), seed)
    if isinstance(dt, T.DateType):
        import datetime as _dt
        days = (v - _dt.date(1970, 1, 1)).days if isinstance(v, _dt.date) else int(v)
        return fi(days, seed)
    if isinstance(dt, T.LongType):
        return fl(int(v), seed)
    if isinstance(dt, T.TimestampType):
        return fl(ts_to_micros(v), seed)
    if isinstance(dt, T.FloatType):
        return fi(_float_bits(float(v)), seed)
    if isinstance(dt, T.DecimalType):
        # Spark: the unscaled value, as a long when precision <= 18, else the two's-complement
        # big-endian bytes of the unscaled BigInteger (BigInteger.toByteArray, minimal length)
        unscaled = _unscaled(v, dt.scale)
        if dt.precision <= 18:
            return fl(unscaled, seed)
        # Java's bitLength ignores the sign bit: for negatives it is that of ~v (-128 -> 7 bits, 1 byte)
        nbits = (unscaled if unscaled >= 0 else ~unscaled).bit_length()
        return fb(unscaled.to_bytes(nbits // 8 + 1, "big", signed=True), seed)
    if isinstance(dt, T.DoubleType):
        return fl(_double_bits(float(v)), seed)
    if isinstance(dt, T.BinaryType):
        return fb(bytes(v), seed)
    if isinstance(dt, T.ArrayType):
        h = seed
        for e in v:
            h = hash_value(e, dt.elementType, h, algo)
        return h
    if isinstance(dt, T.MapType):
        h = seed
        for k, e in v.items():
            h = hash_value(k, dt.keyType, h, algo)
            h = hash_value(e, dt.valueType, h, algo)
        return h
    if isinstance(dt, T.StructType):
        h = seed
        for f, e in zip(dt.fields, v):
            h = hash_value(e, f.dataType, h, algo)
        return h
    return fb(str(v).encode("utf-8"), seed)


# ------------------------------------------------------------------------------------------ device lanes

def _lsr(x: torch.Tensor, s: int) -> torch.Tensor:
    return (x >> s) & ((1 << (64 - s)) - 1)


def _t_rotl32(x, r):
    return ((x << r) | (x >> (32 - r))) & M32


def _t_mixk1(k):
    k = (k * _C1) & M32
    k = _t_rotl32(k, 15)
    return (k * _C2) & M32


def _t_mixh1(h, k):
    h = h ^ k
    h = _t_rotl32(h, 13)
    return (h * 5 + 0xE6546B64) & M32


def _t_fmix32(h, n):
    h = h ^ n
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & M32
    return h ^ (h >> 16)


def _t_rotl64(x, r):
    return (x << r) | _lsr(x, 64 - r)


def _t_xx_fmix(h):
    h = h ^ _lsr(h, 33)
    h = h * _s64(P2)
    h = h ^ _lsr(h, 29)
    h = h * _s64(P3)
    return h ^ _lsr(h, 32)


def device_hash(vals: torch.Tensor, dt: T.DataType, seed: torch.Tensor, algo: str) -> torch.Tensor:
    """Hash a device column (int64 lanes) given per-row seeds; returns the new per-row hash
    (murmur3: uint32 in int64; xxhash64: int64 bit pattern)."""
    if isinstance(dt, (T.FloatType,)):
        f = vals.to(torch.float32) + 0.0
        f = torch.where(torch.isnan(f), torch.full_like(f, float("nan")), f)
        lane, width = f.view(torch.int32).to(torch.int64), 4
    elif isinstance(dt, T.DecimalType):
        if dt.precision > 18:
            raise ValueError("decimal(precision > 18) hashes on the host (unscaled BigInteger bytes)")
        # device decimals are f64: the unscaled long is the value at the column's scale, rounded
        lane, width = torch.round(vals.to(torch.float64) * (10.0 ** dt.scale)).to(torch.int64), 8
    elif isinstance(dt, T.DoubleType):
        f = vals.to(torch.float64) + 0.0
        f = torch.where(torch.isnan(f), torch.full_like(f, float("nan")), f)
        lane, width = f.view(torch.int64), 8
    elif isinstance(dt, (T.LongType, T.TimestampType)):
        lane, width = vals.to(torch.int64), 8
    else:  # boolean / byte / short / int / date
        lane, width = vals.to(torch.int64), 4
    if algo == "murmur3":
        if width == 4:
            return _t_fmix32(_t_mixh1(seed, _t_mixk1(lane & M32)), 4)
        h = _t_mixh1(seed, _t_mixk1(lane & M32))
        h = _t_mixh1(h, _t_mixk1((lane >> 32) & M32))
        return _t_fmix32(h, 8)
    if width == 4:
        h = seed + _s64(P5 + 4)
        h = h ^ ((lane & M32) * _s64(P1))
        h = _t_rotl64(h, 23) * _s64(P2) + _s64(P3)
        return _t_xx_fmix(h)
    h = seed + _s64(P5 + 8)
    h = h ^ (_t_rotl64(lane * _s64(P2), 31) * _s64(P1))
    h = _t_rotl64(h, 27) * _s64(P1) + _s64(P4)
    return _t_xx_fmix(h)


__all__ = ["m3_int", "m3_long", "m3_bytes", "xx_int", "xx_long", "xx_bytes", "hash_value", "device_hash"]
