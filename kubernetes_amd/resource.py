"""resource.Quantity: the fixed-point resource amounts of pkg/api/resource.

Only what the Filter/Score pass consumes at ingest: ParseQuantity
(quantity.go:155-208), Value() / MilliValue() with inf.RoundUp
(quantity.go:335-351), NewQuantity / NewMilliQuantity. Amounts are held
exactly as Fractions (the vendored speter.net/go/exp/math/dec/inf rev 42ca6cd
keeps an unscaled big.Int + scale; both are exact decimals). The reference
converts to int64 once per container per predicate call; here the host does it
once per pod at ingest and the kernels see only the int64 sums.
"""
from __future__ import annotations

import re
from fractions import Fraction

DecimalExponent = "DecimalExponent"
BinarySI = "BinarySI"
DecimalSI = "DecimalSI"

MAX_ALLOWED = (1 << 63) - 1  # quantity.go: maxAllowed == max int64

_SPLIT_RE = re.compile(r"([+-]?[0-9.]+)([eEimkKMGTP]*[-+]?[0-9]*)")

# suffix.go:79-100
_DEC_SUFFIXES = {"m": -3, "": 0, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}
_BIN_SUFFIXES = {"Ki": 10, "Mi": 20, "Gi": 30, "Ti": 40, "Pi": 50, "Ei": 60}


class QuantityError(ValueError):
    pass


def _round_up(x: Fraction, places: int) -> Fraction:
    """inf.Dec.Round(x, places, inf.RoundUp): away from zero (rounder.go:105-125)."""
    scale = 10 ** places
    y = x * scale
    if y.denominator == 1:
        return x
    n = abs(y.numerator) // y.denominator + 1  # magnitude rounded away from zero
    return Fraction(n if y > 0 else -n, scale)


def _ceil_away(n: int, d: int) -> int:
    """n/d (d > 0) rounded away from zero to an integer: _round_up(Fraction(n, d), 0)'s
    numerator in integer arithmetic (ingest calls it per container per pod)."""
    q, r = divmod(abs(n), d)
    q += r != 0
    return q if n >= 0 else -q


def _go_int64(v: int) -> int:
    """big.Int.Int64(): low 64 bits of |v|, negated for v < 0 (two's complement wrap)."""
    mag = abs(v) & ((1 << 64) - 1)
    r = -mag if v < 0 else mag
    r &= (1 << 64) - 1
    return r - (1 << 64) if r >= (1 << 63) else r


def _scan_dec(s: str) -> Fraction:
    """inf.Dec.scan (dec.go:470-518) followed by the must-consume-all check of SetString."""
    unscaled = []
    dp = -1
    dg = -1
    i = 0
    while i < len(s):
        ch = s[i]
        if ch in "+-":
            if unscaled or dp >= 0:
                break
        elif ch == ".":
            if dp >= 0:
                break
            dp = len(unscaled)
            i += 1
            continue
        elif "0" <= ch <= "9":
            if dg == -1:
                dg = len(unscaled)
        else:
            break
        unscaled.append(ch)
        i += 1
    if dg == -1 or i != len(s):
        raise QuantityError(f"unable to parse numeric part of quantity: {s!r}")
    scale = len(unscaled) - dp if dp >= 0 else 0
    u = int("".join(unscaled))
    return Fraction(u, 10 ** scale)


class Quantity:
    __slots__ = ("amount", "format")

    def __init__(self, amount: Fraction, fmt: str = DecimalSI):
        self.amount = Fraction(amount)
        self.format = fmt

    @staticmethod
    def zero() -> "Quantity":
        return Quantity(Fraction(0), DecimalSI)

    @staticmethod
    def from_int(value: int, fmt: str = BinarySI) -> "Quantity":
        """NewQuantity(value, format) (quantity.go:318-324)."""
        return Quantity(Fraction(value), fmt)

    @staticmethod
    def from_milli(value: int, fmt: str = DecimalSI) -> "Quantity":
        """NewMilliQuantity(value, format) (quantity.go:326-333)."""
        return Quantity(Fraction(value, 1000), fmt)

    def value(self) -> int:
        """Value(): Round(0, RoundUp) -> Int64 (quantity.go:335-342)."""
        return _go_int64(_ceil_away(self.amount.numerator, self.amount.denominator))

    def milli_value(self) -> int:
        """MilliValue(): Round(amount*1000, 0, RoundUp) -> Int64 (quantity.go:344-351)."""
        return _go_int64(_ceil_away(self.amount.numerator * 1000, self.amount.denominator))

    def __eq__(self, other):
        return isinstance(other, Quantity) and self.amount == other.amount and self.format == other.format

    def __repr__(self):
        return f"Quantity({self.amount}, {self.format})"


def parse_quantity(s: str) -> Quantity:
    """ParseQuantity (quantity.go:155-208)."""
    m = _SPLIT_RE.fullmatch(s.strip())
    if not m:
        raise QuantityError(f"quantity {s!r} must match ^([+-]?[0-9.]+)([eEimkKMGTP]*[-+]?[0-9]*)$")
    amount = _scan_dec(m.group(1))
    suf = m.group(2)
    if suf in _DEC_SUFFIXES:
        base, exp, fmt = 10, _DEC_SUFFIXES[suf], DecimalSI
    elif suf in _BIN_SUFFIXES:
        base, exp, fmt = 2, _BIN_SUFFIXES[suf], BinarySI
    elif len(suf) > 1 and suf[0] in "eE":
        body = suf[1:]
        if not re.fullmatch(r"[+-]?[0-9]+", body):
            raise QuantityError(f"unable to parse quantity's suffix: {suf!r}")
        exp = int(body)
        if not -(1 << 63) <= exp < (1 << 63):
            raise QuantityError(f"unable to parse quantity's suffix: {suf!r}")
        base, fmt = 10, DecimalExponent
    else:
        raise QuantityError(f"unable to parse quantity's suffix: {suf!r}")
    if base == 10:
        amount = amount * (Fraction(10) ** exp)
    else:
        amount = amount * (1 << exp)
    neg = amount < 0
    if neg:
        amount = -amount
    amount = _round_up(amount, 3)
    if amount > MAX_ALLOWED:
        amount = Fraction(MAX_ALLOWED)
    if fmt == BinarySI and 0 < amount < 1:
        fmt = DecimalSI
    if neg:
        amount = -amount
    return Quantity(amount, fmt)


must_parse = parse_quantity
