"""The numpy RNG algorithms csrc/gen.hip restates, written out in plain Python and pinned against
numpy itself (CPU; the HIP restatement is pinned through the grids it generates, test_gpu_gen.py).

gymnasium's np_random(seed) = Generator(PCG64(SeedSequence(seed))) is how the reference seeds every
env (minigrid_env.py:119-157); its _gen_grid code draws through Generator.integers, .shuffle and
.choice.
"""
import numpy as np
import pytest

M32, M64, M128 = 0xFFFFFFFF, (1 << 64) - 1, (1 << 128) - 1


def seedseq_state(seed):
    ent = []
    n = seed
    if n == 0:
        ent = [0]
    while n > 0:
        ent.append(n & M32)
        n >>= 32
    hc = [0x43b0d7e5]

    def hashmix(v):
        v ^= hc[0]
        hc[0] = (hc[0] * 0x931e8875) & M32
        v = (v * hc[0]) & M32
        return v ^ (v >> 16)

    def mix(x, y):
        r = (0xca01f9dd * x - 0x4973f715 * y) & M32
        return r ^ (r >> 16)

    pool = [hashmix(ent[i] if i < len(ent) else 0) for i in range(4)]
    for s in range(4):
        for d in range(4):
            if s != d:
                pool[d] = mix(pool[d], hashmix(pool[s]))
    for s in range(4, len(ent)):
        for d in range(4):
            pool[d] = mix(pool[d], hashmix(ent[s]))
    h = 0x8b51f9dd
    words = []
    for i in range(8):
        v = pool[i % 4] ^ h
        h = (h * 0x58f38ded) & M32
        v = (v * h) & M32
        words.append(v ^ (v >> 16))
    return [words[2 * i] | (words[2 * i + 1] << 32) for i in range(4)]


class Pcg64:
    MULT = 0x2360ED051FC65DA44385DF649FCCF645

    def __init__(self, seed):
        v = seedseq_state(seed)
        self.inc = ((((v[2] << 64) | v[3]) << 1) | 1) & M128
        self.state = 0
        self._step()
        self.state = (self.state + ((v[0] << 64) | v[1])) & M128
        self._step()
        self.buf = None

    def _step(self):
        self.state = (self.state * self.MULT + self.inc) & M128

    def next64(self):
        self._step()
        hi, lo = self.state >> 64, self.state & M64
        x, rot = hi ^ lo, hi >> 58
        return ((x >> rot) | (x << ((64 - rot) & 63))) & M64

    def next32(self):
        if self.buf is not None:
            b, self.buf = self.buf, None
            return b
        n = self.next64()
        self.buf = n >> 32
        return n & M32

    def integers(self, lo, hi):
        rng = hi - lo - 1
        if rng == 0:
            return lo
        excl = rng + 1
        m = self.next32() * excl
        if (m & M32) < excl:
            thr = (M32 - rng) % excl
            while (m & M32) < thr:
                m = self.next32() * excl
        return lo + (m >> 32)

    def interval(self, mx):
        if mx == 0:
            return 0
        mask = mx
        for s in (1, 2, 4, 8, 16):
            mask |= mask >> s
        while True:
            v = self.next32() & mask
            if v <= mx:
                return v


def _gen(seed):
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


@pytest.mark.parametrize("seed", [0, 1, 2, 123, 65535, 2**31 - 1, 2**32 + 5, 2**40 + 3])
def test_pcg64_raw_stream(seed):
    p = Pcg64(seed)
    assert [int(x) for x in np.random.PCG64(np.random.SeedSequence(seed)).random_raw(8)] == [p.next64() for _ in range(8)]


def test_integers_shuffle_choice_interleaved():
    """One Generator used the way _gen_grid uses it: integers, shuffle and choice interleaved
    (the PCG64 half-word buffer is shared across them)."""
    for seed in range(300):
        G, p = _gen(seed), Pcg64(seed)
        for step in range(6):
            lo, hi = (0, 4) if step % 3 == 0 else (1, 2 + (seed + step) % 17)
            assert int(G.integers(lo, hi)) == p.integers(lo, hi)
            n = 2 + (seed + step) % 7
            a = list(range(n))
            G.shuffle(a)
            b = list(range(n))
            for i in reversed(range(1, n)):
                j = p.interval(i)
                b[i], b[j] = b[j], b[i]
            assert a == b
            c0, c1 = 1 + step, 4 + step + seed % 5
            assert int(G.choice(range(c0, c1))) == c0 + p.integers(0, c1 - c0)
