"""pb_orbit_sum's discrete log (pbgpu_kernels.hip, PB_ORB_LOG12): the payload LCG's 3-step map
M = L^3 mod 2^24 has full period, and the position p of a state y on M's orbit from 0 is found
with its low 12 bits one at a time and its top 12 bits in closed form.  A
Python model of the device arithmetic against the bit-at-a-time walk and against M^p itself."""
import random

A, C = 1103515245, 12345  # glibc rand_r (sequence.c:552-555 draws three steps per payload byte)
M24 = (1 << 24) - 1
A3 = (A * A * A) & M24
C3 = (C * (A * A + A + 1)) & M24


def orb(i):
    """M^(2^i) as (a, c) mod 2^24"""
    a, c = A3, C3
    for _ in range(i):
        c = ((a + 1) * c) & M24
        a = (a * a) & M24
    return a, c


ORB = [orb(i) for i in range(25)]


def log_walk(y):
    cur = p = 0
    for i in range(24):
        a, c = ORB[i]
        if (cur ^ y) >> i & 1:
            cur = (a * cur + c) & M24
            p |= 1 << i
    return p


def log_closed(y):
    cur = p = 0
    for i in range(12):
        a, c = ORB[i]
        if (cur ^ y) >> i & 1:
            cur = (a * cur + c) & M24
            p |= 1 << i
    a12, c12 = ORB[12]
    w = ((y & 0xFFF) * ((a12 - 1) >> 12) + (c12 >> 12)) & 0xFFF
    x = w
    for _ in range(2):
        x = (x * ((2 - w * x) & 0xFFF)) & 0xFFF
    j = ((((y - cur) & M24) >> 12) * x) & 0xFFF
    return p | (j << 12)


def power(x, p):
    for i in range(24):
        if p >> i & 1:
            a, c = ORB[i]
            x = (a * x + c) & M24
    return x


def test_shape_of_m_4096():
    a12, c12 = ORB[12]
    assert (a12 - 1) % (1 << 14) == 0 and c12 % (1 << 12) == 0 and (c12 >> 12) & 1


def test_closed_form_matches_the_walk():
    rng = random.Random(7)
    ys = [0, 1, M24, 1 << 12, (1 << 12) - 1] + [rng.randrange(1 << 24) for _ in range(4000)]
    for y in ys:
        p = log_closed(y)
        assert p == log_walk(y), y
        assert power(0, p) == y, y
