"""The FASTA tile pass counts a mask word's candidates by carries (SIDX_FA_CARRY,
shock_amd/csrc/sidx_kernels.hip fa_iter): a '>' is a candidate (fasta.go:100-138) iff the marker
('>' or '\\n') nearest below it is a '\\n'.  This checks the bit identity against the loop it
replaced (one iteration per '>', the previous '\\n' / '>' looked up per bit) on random words,
including the carry-in from earlier words (NLx / GTx: the last '\\n' / '>' + 1 before the word in
the wave, 0 if none) and the conditional first '>' of a wave."""
import random

M = (1 << 64) - 1


def by_loop(nl, gt, NLx, GTx, base):
    c = cond = 0
    pg = GTx
    m = gt
    while m:
        j = (m & -m).bit_length() - 1
        m &= m - 1
        nb = nl & ((1 << j) - 1)
        pn = base + nb.bit_length() if nb else NLx
        if pg == 0 and pn == 0:
            cond = 1
        elif pg == 0 or pn > pg:
            c += 1
        pg = base + j + 1
    return c, cond


def by_carry(nl, gt, NLx, GTx):
    u = nl | gt
    s = ((~u & M) + ((nl << 1) & M) + (1 if NLx > GTx else 0)) & M
    cond = 1 if (GTx == 0 and NLx == 0 and (u & (-u & M) & gt)) else 0
    return bin(gt & s).count("1"), cond


def test_carry_count_matches_loop():
    rng = random.Random(0x5EED)
    for _ in range(40000):
        d = rng.choice([0.02, 0.1, 0.3, 0.6, 0.95])
        nl = gt = 0
        for b in range(64):
            r = rng.random()
            if r < d / 2:
                nl |= 1 << b
            elif r < d:
                gt |= 1 << b
        base = 64 * rng.randint(1, 63)
        GTx = rng.choice([0, rng.randint(1, base)])
        NLx = rng.choice([0, rng.randint(1, base)])
        assert by_loop(nl, gt, NLx, GTx, base) == by_carry(nl, gt, NLx, GTx), (hex(nl), hex(gt), NLx, GTx)


def test_carry_count_edges():
    base = 128
    for nl, gt in [(0, 0), (0, M), (M, 0), (1, 2), (2, 1), (1 << 63, 1), (1, 1 << 63),
                   (0x5555555555555555, 0xAAAAAAAAAAAAAAAA), (0xAAAAAAAAAAAAAAAA, 0x5555555555555555)]:
        for NLx, GTx in [(0, 0), (5, 0), (0, 5), (5, 7), (7, 5)]:
            assert by_loop(nl, gt, NLx, GTx, base) == by_carry(nl, gt, NLx, GTx)
