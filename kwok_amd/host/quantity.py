"""k8s.io/apimachinery v0.30.2 ``resource.ParseQuantity`` + ``AsApproximateFloat64``.

The usage evaluator turns every container's usage into a float64 through
``Quantity.AsApproximateFloat64`` (metrics_resource_usage.go:148, cel/environment.go:133 for
CEL ``Quantity(...)`` results).  apimachinery is a dependency absent from /root/reference
(go.mod: k8s.io/apimachinery v0.30.2); this restates its published algorithm
(api/resource/quantity.go: parseQuantityString, ParseQuantity, AsApproximateFloat64; and
Go's math.Pow10).  The host parses each distinct quantity string once and hands the device
interned float64 values.
"""
from __future__ import annotations

from fractions import Fraction
from typing import Optional

import numpy as np

_DEC = {"n": -9, "u": -6, "m": -3, "": 0, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}
_BIN = {"Ki": 10, "Mi": 20, "Gi": 30, "Ti": 40, "Pi": 50, "Ei": 60}
_MAX_INT64_FACTORS = 18
INT64_MAX = (1 << 63) - 1

_POW10TAB = [float(f"1e{i}") for i in range(32)]
_POW10POSTAB32 = [float(f"1e{32 * i}") for i in range(10)]
_POW10NEGTAB32 = [float(f"1e-{32 * i}") for i in range(11)]


def go_pow10(n: int) -> float:
    """math.Pow10 (Go 1.22)."""
    if 0 <= n <= 308:
        return _POW10POSTAB32[n // 32] * _POW10TAB[n % 32]
    if -323 <= n <= 0:
        return _POW10NEGTAB32[(-n) // 32] / _POW10TAB[(-n) % 32]
    return float("inf") if n > 0 else 0.0


class QuantityError(ValueError):
    pass


def _parse_quantity_string(s: str):
    positive = True
    pos = 0
    end = len(s)
    if pos < end:
        if s[0] == "-":
            positive = False
            pos += 1
        elif s[0] == "+":
            pos += 1
    i = pos
    while True:  # strip leading zeros
        if i >= end:
            return positive, "0", "0", "", ""
        if s[i] == "0":
            pos += 1
            i += 1
        else:
            break
    i = pos
    while True:
        if i >= end:
            return positive, s[0:end], s[pos:end], "", ""
        if "0" <= s[i] <= "9":
            i += 1
            continue
        num = s[pos:i]
        pos = i
        break
    if len(num) == 0:
        num = "0"
    denom = ""
    if pos < end and s[pos] == ".":
        pos += 1
        i = pos
        while True:
            if i >= end:
                return positive, s[0:end], num, s[pos:end], ""
            if "0" <= s[i] <= "9":
                i += 1
                continue
            denom = s[pos:i]
            pos = i
            break
    value = s[0:pos]
    suffix_start = pos
    i = pos
    while True:
        if i >= end:
            return positive, value, num, denom, s[suffix_start:end]
        if s[i] not in "eEinumkKMGTP":
            pos = i
            break
        i += 1
    if pos < end and s[pos] in "-+":
        pos += 1
    i = pos
    while True:
        if i >= end:
            return positive, value, num, denom, s[suffix_start:end]
        if "0" <= s[i] <= "9":
            i += 1
            continue
        raise QuantityError("quantities must match the regular expression")


def _interpret(suf: str):
    if suf in _DEC:
        return 10, _DEC[suf], "DecimalSI"
    if suf in _BIN:
        return 2, _BIN[suf], "BinarySI"
    if len(suf) > 1 and suf[0] in "eE":
        body = suf[1:]
        try:
            if not body or not all(c in "+-0123456789" for c in body) or "+" in body[1:] or "-" in body[1:]:
                raise ValueError
            e = int(body, 10)
        except ValueError:
            raise QuantityError("unable to parse quantity's suffix")
        if not (-(1 << 63) <= e < (1 << 63)):
            raise QuantityError("unable to parse quantity's suffix")
        return 10, ((e + (1 << 31)) % (1 << 32)) - (1 << 31), "DecimalExponent"  # int32(parsed)
    raise QuantityError("unable to parse quantity's suffix")


def _round_up_to_nano(x: Fraction) -> Fraction:
    scaled = x * 10**9
    n = scaled.numerator // scaled.denominator
    if n != scaled:  # RoundUp = away from zero for the magnitude (x >= 0 here)
        n += 1
    return Fraction(n, 10**9)


def parse_quantity_f64(s: str) -> float:
    """ParseQuantity(s).AsApproximateFloat64(); raises QuantityError when ParseQuantity fails."""
    if len(s) == 0:
        raise QuantityError("quantities must match the regular expression")
    if s == "0":
        return 0.0
    positive, value, num, denom, suf = _parse_quantity_string(s)
    base, exponent, fmt = _interpret(suf)
    precision = 0
    scale = 0
    mantissa = 1
    if fmt in ("DecimalExponent", "DecimalSI"):
        scale = exponent
        precision = _MAX_INT64_FACTORS - (len(num) + len(denom))
    else:
        scale = 0
        if exponent >= 0 and len(denom) == 0:
            mantissa = 1 << exponent
            # int32(float32(exponent)*3/10): float32 arithmetic then truncation toward zero
            precision = 15 - len(num) - int(np.float32(exponent) * np.float32(3) / np.float32(10)) - 1
        else:
            precision = -1
    if precision >= 0:
        scale -= len(denom)
        if scale >= -9:
            shifted = num + denom
            v = int(shifted, 10)
            if v > INT64_MAX:
                raise QuantityError("quantities must match the regular expression")
            result = v * mantissa
            if -(1 << 63) <= result <= INT64_MAX:  # int64Multiply ok
                if not positive:
                    result = -result
                # int64Amount{value: result, scale}
                if scale == 0:
                    return float(result)
                return float(result) * go_pow10(scale)
    # inf.Dec path
    try:
        amount = Fraction(value) if value not in ("", "+", "-") else None
    except (ValueError, ZeroDivisionError):
        amount = None
    if amount is None:
        raise QuantityError("quantities must match the regular expression")
    if base == 10:
        amount = amount * (Fraction(10) ** exponent)
    else:
        amount = amount * (1 << exponent)
    sign = -1 if amount < 0 else 1
    amount = abs(amount)
    if amount != 0:
        amount = _round_up_to_nano(amount)
    if fmt == "BinarySI" and amount > INT64_MAX:
        amount = Fraction(INT64_MAX)
    amount = amount * sign
    # AsApproximateFloat64 of the inf.Dec: unscaled big int -> float64, times Pow10(-scale).
    # After rounding to nano the decimal has scale 9 (or less if exact with fewer digits: inf.Dec
    # keeps scale 9 after Round).
    scale_d = 9 if amount != 0 else _dec_scale(value, base, exponent)
    unscaled = amount * (10**scale_d)
    assert unscaled.denominator == 1
    b = float(int(unscaled))  # big.Float.SetInt(...).Float64(): round half to even == Python int->float
    e = -scale_d
    if e == 0:
        return b
    return b * go_pow10(e)


def _dec_scale(value: str, base: int, exponent: int) -> int:
    frac = value.split(".", 1)[1] if "." in value else ""
    return len(frac) - (exponent if base == 10 else 0)


def parse_quantity_or_none(s: str) -> Optional[float]:
    try:
        return parse_quantity_f64(s)
    except QuantityError:
        return None
