"""CPU model of kmeans.hip ordered_sum_wave (the binade-segmented scan that
replaces the sequential cluster-0 sum): the same steps in Python doubles,
checked against the plain left-to-right sum on random, sign-changing,
tie-heavy and extreme inputs.  Run: python tools/probe/km_scan_model.py"""
import math
import os
import random
import sys

P = int(os.environ.get("KML_SCAN_PER", "4"))  # elements per lane per step
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
        bigm = [0] * W
        tiem = [0] * W
        tot = [0.0] * W
        for l in range(W):
            run = 0.0
            for k in range(P):
                X = ldexp(sg * x[l][k], 53 - e)
                big = not (abs(X) < 2.0 ** 51)
                tie = (not big) and (X - math.floor(X)) == 0.5
                bigm[l] |= int(big) << k
                tiem[l] |= int(tie) << k
                # a tie counts its lower neighbour floor(X); the parity pass below adds 1 when it rounds up
                run = run + (0.0 if big else (float(math.floor(X)) if tie else rint(X)))
                L[l][k] = run
            tot[l] = run
        E = [0.0] * W
        s = 0.0
        for l in range(W):
            E[l] = s
            s = s + tot[l]
        T = [[A + (E[l] + L[l][k]) for k in range(P)] for l in range(W)]
        # hard exits: large elements or prefixes near the binade ends (a margin of
        # MARGIN grid steps absorbs the tie corrections, at most MAXTIE of them)
        MARGIN, MAXTIE = 64, 32
        fh = c
        for l in range(W):
            kl = min(max(c - P * l, 0), P)
            for k in range(kl):
                if ((bigm[l] >> k) & 1) or not (2.0 ** 52 + MARGIN <= T[l][k] <= 2.0 ** 53 - MARGIN):
                    fh = min(fh, P * l + k)
        # ties before the first hard exit, in order: round half to even
        nt = 0
        for q in range(fh):
            l, k = divmod(q, P)
            if (tiem[l] >> k) & 1:
                if nt == MAXTIE:
                    fh = q  # too many: this tie is added for real
                    break
                nt += 1
                stats["ties"] += 1
                if int(T[l][k]) & 1:
                    for p2 in range(q, W * P):
                        l2, k2 = divmod(p2, P)
                        T[l2][k2] += 1.0
        if fh == c:
            ll, kk = (c - 1) // P, (c - 1) % P
            acc = sg * ldexp(T[ll][kk], e - 53)
            i += c
        else:
            lf, fk = divmod(fh, P)
            Tpre = A if fh == 0 else T[(fh - 1) // P][(fh - 1) % P]
            acc = sg * ldexp(Tpre, e - 53)
            acc = acc + x[lf][fk]
            f = fh
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
    st = {"steps": 0, "exits": 0, "seq": 0, "ties": 0}
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
    print(f"ok: {cases} cases, {st['steps']} steps, {st['exits']} exits, {st['ties']} ties in-scan, "
          f"{st['seq']} sequential elements")
    return 0


if __name__ == "__main__":
    sys.exit(main())
