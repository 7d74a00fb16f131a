"""java.util.Random, as far as ErasureCodeTest uses it (seeded constructor +
nextBytes).  The JDK specifies the algorithm exactly (48-bit LCG, multiplier
0x5DEECE66D, addend 0xB), so the reference test's inputs
(ErasureCodeTest.java:34, :61, :69) can be regenerated without a JVM."""
import numpy as np

_MULT = 0x5DEECE66D
_ADD = 0xB
_MASK = (1 << 48) - 1


class JavaRandom:
    def __init__(self, seed: int):
        self.seed = (seed ^ _MULT) & _MASK

    def _next(self, bits: int) -> int:
        self.seed = (self.seed * _MULT + _ADD) & _MASK
        r = self.seed >> (48 - bits)
        if r >= 1 << (bits - 1):  # to signed int32 for bits == 32
            r -= 1 << bits
        return r

    def nextInt(self) -> int:
        return self._next(32)

    def nextBytes(self, n: int) -> np.ndarray:
        """Random.nextBytes: 4 bytes per nextInt(), low byte first."""
        out = np.empty(n, np.uint8)
        i = 0
        while i < n:
            rnd = self.nextInt() & 0xFFFFFFFF
            for _ in range(min(n - i, 4)):
                out[i] = rnd & 0xFF
                rnd >>= 8
                i += 1
        return out
