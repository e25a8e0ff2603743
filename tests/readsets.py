"""Deterministic read sets covering the edge cases BaseAligner::AlignRead handles
(BaseAligner.cpp:582-938): exact / mutated / indel reads in both orientations,
reads with Ns (up to and past maxK), shorter than a seed, long reads, lower-case
and IUPAC bytes, contig ends, repeat copies (popular seeds), palindromic seeds,
random reads and assorted quality strings."""
import random

COMP = {"A": "T", "C": "G", "G": "C", "T": "A", "N": "N"}


def revcomp(s):
    return "".join(COMP.get(c, "N") for c in reversed(s))


def _quals(rng, n, kind):
    if kind == 0:
        return "2" * n                      # wgsim Q17
    if kind == 1:
        return "".join(chr(33 + rng.randrange(0, 42)) for _ in range(n))
    if kind == 2:
        return "I" * n
    return "".join(chr(33 + rng.choice([2, 10, 20, 30, 40])) for _ in range(n))


def _mutate(rng, s, nsub, nindel):
    s = list(s)
    for _ in range(nsub):
        i = rng.randrange(len(s))
        s[i] = rng.choice([b for b in "ACGT" if b != s[i]])
    for _ in range(nindel):
        i = rng.randrange(1, len(s) - 1)
        if rng.random() < 0.5:
            del s[i]
        else:
            s.insert(i, rng.choice("ACGT"))
    return "".join(s)


def edge_reads(genome, n_random=400, seed=7, max_len=500):
    """genome: snapgpu.Genome (or anything with .n_bases / .bases(start, len) / .pieces)."""
    rng = random.Random(seed)
    nb = genome.n_bases
    pieces = genome.pieces
    pad = pieces[0][1] if pieces else 500
    out = []

    def sub(start, length):
        return genome.bases(start, length).decode().replace("n", "N")

    def rand_pos(length):
        for _ in range(100):
            p = rng.randrange(pad, nb - pad - length)
            s = sub(p, length)
            if s.count("N") == 0:
                return p, s
        return p, s

    for i in range(n_random):
        L = rng.choice([100, 100, 100, 101, 75, 150])
        p, s = rand_pos(L)
        kind = i % 8
        if kind == 1:
            s = _mutate(rng, s, rng.randrange(1, 6), 0)
        elif kind == 2:
            s = _mutate(rng, s, rng.randrange(0, 3), rng.randrange(1, 4))
        elif kind == 3:
            s = _mutate(rng, s, rng.randrange(6, 20), rng.randrange(0, 2))
        elif kind == 4:
            s = list(s)
            for _ in range(rng.choice([1, 3, 14, 15, 20])):
                s[rng.randrange(len(s))] = "N"
            s = "".join(s)
        if rng.random() < 0.5:
            s = revcomp(s)
        out.append((s, _quals(rng, len(s), i % 4)))
    # contig boundaries (reads overlapping padding) and the very first / last bases
    for name, off in pieces:
        for delta in (-60, -20, 0, 5, 40):
            st = off + delta
            if 0 <= st < nb - 200:
                s = sub(st, 100)
                out.append((s, _quals(rng, 100, 0)))
                out.append((revcomp(s), _quals(rng, 100, 1)))
    # length edge cases
    for L in (1, 10, 19, 20, 21, 22, 39, 40, 41, 50, 64, 65, 99, 127, 128, 129, 200, 250, 300, 499, 500):
        if L > max_len:
            continue
        p, s = rand_pos(L)
        out.append((s, _quals(rng, L, 1)))
        out.append((revcomp(_mutate(rng, s, 1 if L > 30 else 0, 0)), _quals(rng, L, 0)))
    # lower-case and IUPAC bytes (Read::init upper-cases; non-ACGTN complement to 0)
    for _ in range(12):
        p, s = rand_pos(100)
        out.append((s.lower(), _quals(rng, 100, 0)))
        t = list(s)
        for _ in range(3):
            t[rng.randrange(100)] = rng.choice("RYKMSW")
        out.append(("".join(t), _quals(rng, 100, 1)))
    # random reads, homopolymers, palindromic seeds
    for _ in range(20):
        out.append(("".join(rng.choice("ACGT") for _ in range(100)), _quals(rng, 100, 0)))
    out.append(("A" * 100, "I" * 100))
    out.append(("T" * 100, "I" * 100))
    out.append(("ACGT" * 25, "2" * 100))
    out.append(("AATT" * 25, "2" * 100))
    out.append(("GATC" * 25, "5" * 100))
    out.append(("N" * 100, "2" * 100))
    # quality-string extremes
    for qc in ("!", "#", "~"):
        p, s = rand_pos(100)
        out.append((_mutate(rng, s, 3, 1), qc * len(s)))
    return out
