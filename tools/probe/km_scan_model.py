"""CPU model of kmeans.hip ordered_sum_wave (the binade-segmented scan that
replaces the sequential cluster-0 sum): the same steps in Python doubles,
checked against the plain left-to-right sum on random, sign-changing,
tie-heavy and extreme inputs.  Run: python tools/probe/km_scan_model.py"""
import math
import random
import sys

P = 4   # elements per lane per step
W = 64  # lanes


def seq_sum(acc, xs):
    for x in xs:
        acc = acc + x
    return acc


def ldexp(x, e):
    try:
        return math.ldexp(x, e)
    except OverflowError:
        return math.copysign(math.inf, x)


def frexp_exp(x):
    return math.frexp(x)[1]


def rint(x):
    return float(round(x)) if math.isfinite(x) else x


def wave_sum(acc, xs, stats):
    n = len(xs)
    i = 0
    seq = 0
    while i < n:
        stats["steps"] += 1
        c = min(W * P, n - i)
        x = [[(xs[i + P * l + k] if i + P * l + k < n else 0.0) for k in range(P)] for l in range(W)]
        if seq > 0 or not (acc != 0.0 and math.isfinite(acc)):
            mm = min(seq, c) if seq > 0 else 1
            for j in range(mm):
                acc = acc + x[j // P][j % P]
            seq = seq - mm if seq > 0 else 0
            i += mm
            stats["seq"] += mm
            continue
        e = frexp_exp(acc)
        sg = -1.0 if acc < 0.0 else 1.0
        A = ldexp(abs(acc), 53 - e)
        L = [[0.0] * P for _ in range(W)]
        badm = [0] * W
        tot = [0.0] * W
        for l in range(W):
            run = 0.0
            for k in range(P):
                X = ldexp(sg * x[l][k], 53 - e)
                bad = not (abs(X) < 2.0 ** 51) or (X - math.floor(X)) == 0.5
                badm[l] |= int(bad) << k
                run = run + (0.0 if bad else rint(X))
                L[l][k] = run
            tot[l] = run
        # exclusive scan (exact for lanes up to the first exit in the model as on the GPU)
        E = [0.0] * W
        s = 0.0
        for l in range(W):
            E[l] = s
            s = s + tot[l]
        outm = [0] * W
        for l in range(W):
            kl = min(max(c - P * l, 0), P)
            for k in range(P):
                T = A + (E[l] + L[l][k])
                out = k < kl and (((badm[l] >> k) & 1) or not (2.0 ** 52 + 1 <= T <= 2.0 ** 53 - 1))
                outm[l] |= int(out) << k
        lanes = [l for l in range(W) if outm[l]]
        if not lanes:
            ll, kk = (c - 1) // P, (c - 1) % P
            acc = sg * ldexp(A + (E[ll] + L[ll][kk]), e - 53)
            i += c
        else:
            lf = lanes[0]
            fk = (outm[lf] & -outm[lf]).bit_length() - 1
            Tpre = A + E[lf] if fk == 0 else A + (E[lf] + L[lf][fk - 1])
            acc = sg * ldexp(Tpre, e - 53)
            acc = acc + x[lf][fk]
            f = P * lf + fk
            i += f + 1
            stats["exits"] += 1
            if f < 16:
                seq = 32
    return acc


def same(a, b):
    return (math.isnan(a) and math.isnan(b)) or (a == b and math.copysign(1, a) == math.copysign(1, b))


def check(seed=1, trials=3000):
    """Returns (cases, stats) or raises AssertionError on the first mismatch."""
    rnd = random.Random(seed)
    cases = 0
    st = {"steps": 0, "exits": 0, "seq": 0}
    for trial in range(trials):
        kind = trial % 6
        n = rnd.choice([0, 1, 5, 63, 64, 65, 255, 256, 257, 286, 600, 1300])
        if kind == 0:    # k-means like: mean + noise
            mu = rnd.uniform(-1, 1)
            xs = [mu + rnd.gauss(0, 0.6) for _ in range(n)]
        elif kind == 1:  # zero mean: the sum random-walks across binades and signs
            xs = [rnd.gauss(0, 1) for _ in range(n)]
        elif kind == 2:  # coarse dyadic values: ties everywhere
            xs = [rnd.randint(-64, 64) / 8.0 for _ in range(n)]
        elif kind == 3:  # wide magnitudes
            xs = [rnd.choice([-1, 1]) * 2.0 ** rnd.randint(-60, 60) * rnd.random() for _ in range(n)]
        elif kind == 4:  # same sign, growing
            xs = [abs(rnd.gauss(0.7, 0.3)) for _ in range(n)]
        else:            # specials sprinkled in
            xs = [rnd.gauss(0, 1) for _ in range(n)]
            for _ in range(rnd.randint(0, 3)):
                if n:
                    xs[rnd.randrange(n)] = rnd.choice([0.0, -0.0, 1e300, -1e300, 5e-324, math.inf, 2.0 ** -1074 * 3])
        acc0 = rnd.choice([0.0, 0.0, rnd.gauss(0, 100), rnd.gauss(0, 1e6), -0.0, 2.0 ** 52])
        a = seq_sum(acc0, xs)
        b = wave_sum(acc0, xs, st)
        assert same(a, b), ("mismatch", trial, kind, n, acc0, a, b)
        cases += 1
    return cases, st


def main():
    cases, st = check(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
    print(f"ok: {cases} cases, {st['steps']} steps, {st['exits']} exits, {st['seq']} sequential elements")
    return 0


if __name__ == "__main__":
    sys.exit(main())
