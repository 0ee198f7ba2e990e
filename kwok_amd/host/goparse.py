"""Go parsing semantics the value getters rely on, evaluated host-side at ingest.

The device never parses strings: the host pre-parses each distinct ``weightFrom`` /
``durationFrom`` / ``jitterDurationFrom`` result into an (kind, int64) value record.
Restated from Go 1.22 (the reference's toolchain, go.mod:3):
  strconv.ParseInt(s, 0, 0)   (expression/value_int_from.go:69)
  time.ParseDuration          (expression/value_duration_from.go:73)
  time.Parse(RFC3339Nano, s)  (expression/value_duration_from.go:68)
"""
from __future__ import annotations

import calendar
from typing import Optional, Tuple

INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1


def _lower(c: str) -> str:
    return c.lower() if "A" <= c <= "Z" else c


def _underscore_ok(s: str) -> bool:
    saw = "^"
    i = 0
    if s and s[0] in "+-":
        s = s[1:]
    hexa = False
    if len(s) >= 2 and s[0] == "0" and _lower(s[1]) in "box":
        i = 2
        saw = "0"
        hexa = _lower(s[1]) == "x"
    while i < len(s):
        c = s[i]
        if "0" <= c <= "9" or (hexa and "a" <= _lower(c) <= "f"):
            saw = "0"
        elif c == "_":
            if saw != "0":
                return False
            saw = "_"
        else:
            if saw == "_":
                return False
            saw = "!"
        i += 1
    return saw != "_"


def parse_int(s: str) -> Optional[int]:
    """strconv.ParseInt(s, 0, 0) on 64-bit; None on any error."""
    if not s:
        return None
    neg = False
    body = s
    if body[0] == "+":
        body = body[1:]
    elif body[0] == "-":
        neg = True
        body = body[1:]
    if not body:
        return None
    s0 = body
    base = 10
    if body[0] == "0":
        if len(body) >= 3 and _lower(body[1]) == "b":
            base, body = 2, body[2:]
        elif len(body) >= 3 and _lower(body[1]) == "o":
            base, body = 8, body[2:]
        elif len(body) >= 3 and _lower(body[1]) == "x":
            base, body = 16, body[2:]
        else:
            base, body = 8, body[1:]
    n = 0
    underscores = False
    for c in body:
        if c == "_":
            underscores = True
            continue
        if "0" <= c <= "9":
            d = ord(c) - 48
        elif "a" <= _lower(c) <= "z":
            d = ord(_lower(c)) - ord("a") + 10
        else:
            return None
        if d >= base:
            return None
        n = n * base + d
        if n > (1 << 64) - 1:
            return None  # range error
    if underscores and not _underscore_ok(s0):
        return None
    if not neg and n >= 1 << 63:
        return None
    if neg and n > 1 << 63:
        return None
    return -n if neg else n


_UNITS = {"ns": 1, "us": 1000, "µs": 1000, "μs": 1000, "ms": 10**6, "s": 10**9, "m": 60 * 10**9,
          "h": 3600 * 10**9}


def parse_duration(orig: str) -> Optional[int]:
    """time.ParseDuration; None on error."""
    s = orig
    d = 0
    neg = False
    lim = 1 << 63
    if s and s[0] in "+-":
        neg = s[0] == "-"
        s = s[1:]
    if s == "0":
        return 0
    if not s:
        return None
    while s:
        if not (s[0] == "." or "0" <= s[0] <= "9"):
            return None
        i = 0
        v = 0
        while i < len(s) and "0" <= s[i] <= "9":
            if v > lim // 10:
                return None
            v = v * 10 + ord(s[i]) - 48
            if v > lim:
                return None
            i += 1
        pre = i > 0
        s = s[i:]
        post = False
        f, scale = 0, 1.0
        if s and s[0] == ".":
            s = s[1:]
            j = 0
            overflow = False
            while j < len(s) and "0" <= s[j] <= "9":
                if not overflow:
                    if f > (lim - 1) // 10:
                        overflow = True
                    else:
                        y = f * 10 + ord(s[j]) - 48
                        if y > lim:
                            overflow = True
                        else:
                            f = y
                            scale *= 10
                j += 1
            post = j > 0
            s = s[j:]
        if not pre and not post:
            return None
        k = 0
        while k < len(s) and not (s[k] == "." or "0" <= s[k] <= "9"):
            k += 1
        if k == 0:
            return None
        unit = _UNITS.get(s[:k])
        s = s[k:]
        if unit is None:
            return None
        if v > lim // unit:
            return None
        v *= unit
        if f > 0:
            v += int(float(f) * (float(unit) / scale))
            if v > lim:
                return None
        d += v
        if d > lim:
            return None
    if neg:
        return -d
    if d > lim - 1:
        return None
    return d


def _days_in(m: int, y: int) -> int:
    if m == 2:
        return 29 if (y % 4 == 0 and (y % 100 != 0 or y % 400 == 0)) else 28
    return [31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31][m - 1]


def _digits(s, pos, n) -> Optional[int]:
    part = s[pos:pos + n]
    if len(part) != n or not all("0" <= c <= "9" for c in part):
        return None
    return int(part)


def _nanos(frac_with_sep: str, nbytes: int) -> int:
    nbytes = min(nbytes, 10)
    ns = int(frac_with_sep[1:nbytes])
    return ns * 10 ** (10 - nbytes)


def _epoch(y, mo, d, h, mi, se, zone) -> int:
    # proleptic Gregorian day count from 1970-01-01 (valid for year 0..9999)
    yy = y - (1 if mo <= 2 else 0)
    era = yy // 400
    yoe = yy - era * 400
    doy = (153 * (mo + (-3 if mo > 2 else 9)) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    days = era * 146097 + doe - 719468
    return days * 86400 + h * 3600 + mi * 60 + se - zone


def parse_rfc3339nano(s: str) -> Optional[Tuple[int, int]]:
    """time.Parse(time.RFC3339Nano, s) -> (unix seconds, nanoseconds) or None."""
    r = _fast(s)
    return r if r is not None else _generic(s)


def _fast(s):
    if len(s) < 19:
        return None
    vals = [_digits(s, 0, 4), _digits(s, 5, 2), _digits(s, 8, 2), _digits(s, 11, 2), _digits(s, 14, 2),
            _digits(s, 17, 2)]
    if any(v is None for v in vals):
        return None
    y, mo, d, h, mi, se = vals
    if not (1 <= mo <= 12) or not (1 <= d <= _days_in(mo, y)) or h > 23 or mi > 59 or se > 59:
        return None
    if not (s[4] == "-" and s[7] == "-" and s[10] == "T" and s[13] == ":" and s[16] == ":"):
        return None
    rest = s[19:]
    ns = 0
    if len(rest) >= 2 and rest[0] == "." and "0" <= rest[1] <= "9":
        n = 2
        while n < len(rest) and "0" <= rest[n] <= "9":
            n += 1
        ns = _nanos(rest, n)
        rest = rest[n:]
    zone = 0
    if rest != "Z":
        if len(rest) != 6:
            return None
        hr, mm = _digits(rest, 1, 2), _digits(rest, 4, 2)
        if hr is None or mm is None or hr > 23 or mm > 59:
            return None
        if rest[0] not in "+-" or rest[3] != ":":
            return None
        zone = (hr * 60 + mm) * 60 * (-1 if rest[0] == "-" else 1)
    return _epoch(y, mo, d, h, mi, se, zone), ns


def _generic(v):
    p = 0
    y = _digits(v, p, 4)
    if y is None:
        return None
    p += 4
    if v[p:p + 1] != "-":
        return None
    p += 1
    mo = _digits(v, p, 2)
    if mo is None:
        return None
    p += 2
    if v[p:p + 1] != "-":
        return None
    p += 1
    d = _digits(v, p, 2)
    if d is None:
        return None
    p += 2
    if v[p:p + 1] != "T":
        return None
    p += 1
    if not (p < len(v) and "0" <= v[p] <= "9"):
        return None
    h = ord(v[p]) - 48
    p += 1
    if p < len(v) and "0" <= v[p] <= "9":
        h = h * 10 + ord(v[p]) - 48
        p += 1
    if v[p:p + 1] != ":":
        return None
    p += 1
    mi = _digits(v, p, 2)
    if mi is None:
        return None
    p += 2
    if v[p:p + 1] != ":":
        return None
    p += 1
    se = _digits(v, p, 2)
    if se is None:
        return None
    p += 2
    ns = 0
    if p + 1 < len(v) and v[p] in ".," and "0" <= v[p + 1] <= "9":
        i = 0
        while p + i + 1 < len(v) and "0" <= v[p + i + 1] <= "9":
            i += 1
        ns = _nanos(v[p:], 1 + i)
        p += 1 + i
    zone = 0
    if v[p:p + 1] == "Z":
        p += 1
    else:
        if len(v) - p < 6 or v[p + 3] != ":":
            return None
        hr, mm = _digits(v, p + 1, 2), _digits(v, p + 4, 2)
        if hr is None or mm is None or hr > 24 or mm > 60 or v[p] not in "+-":
            return None
        zone = (hr * 60 + mm) * 60 * (-1 if v[p] == "-" else 1)
        p += 6
    if p != len(v):
        return None
    if not (1 <= mo <= 12) or h >= 24 or mi >= 60 or se >= 60 or not (1 <= d <= _days_in(mo, y)):
        return None
    return _epoch(y, mo, d, h, mi, se, zone), ns


def time_sub(t: Tuple[int, int], now_ns: int) -> int:
    """time.Time.Sub with saturation."""
    d = t[0] * 10**9 + t[1] - now_ns
    return max(INT64_MIN, min(INT64_MAX, d))


def f64_to_i64(x: float) -> int:
    """Go int64(float64) on amd64 (CVTTSD2SQ): NaN / out of range -> INT64_MIN."""
    if x != x or not (-9223372036854775808.0 <= x < 9223372036854775808.0):
        return INT64_MIN
    return int(x)
