"""Sequential chained-beacon stores for the replay workload — bench / test data only.

A replay checks round k against the STORED signature of round k-1 (chain/boltdb/trimmed.go:183): with a
store holding sigma_1..sigma_n, round k verifies iff sigma_k = [sk] H(SHA-256(sigma_{k-1} || k)) (sigma_0 = the
genesis seed). Corrupting sigma_k therefore fails round k and round k+1 (core/drand_test.go:1105-1111).

Signing such a chain is serial (each message needs the previous signature), so it is cut at the corrupted
rounds: the rounds after corruption k_j form segment j, and every segment is signed round by round, all segments
side by side in one device batch per step (dh_sign_batch). The first round of a segment (round k_j + 1) is signed
over a random 96-byte "previous signature": the store hands the verifier the corrupted sigma_{k_j} instead, so
round k_j + 1 fails exactly as it does in a real chain whose sigma_{k_j} was corrupted after the fact (either way
its signature is a valid signature of a message the verifier cannot reproduce). Every other round is a real link:
prev = the stored signature of the round before. Steps = the longest segment.
"""
import numpy as np

import g2_synth

MASK64 = (1 << 64) - 1


def splitmix64(state):
    state = (state + 0x9E3779B97F4A7C15) & MASK64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return state, z ^ (z >> 31)


def corrupted_rounds(n, count, seed=0xD5A11D):
    """Cfg5: `count` distinct 0-based round indices in [0, n) drawn with splitmix64(seed), ascending."""
    st, out = seed, set()
    while len(out) < count:
        st, z = splitmix64(st)
        out.add(z % n)
    return np.array(sorted(out), dtype=np.int64)


def sign_chain(scheme, sk, first_round, n, genesis_seed, breaks, rng, progress=None):
    """Signatures (n, 96) of rounds first_round .. first_round+n-1 chained on their predecessors, cut after each
    index in `breaks` (the rounds that will be corrupted). Row 0's previous signature is `genesis_seed`."""
    starts = np.unique(np.concatenate([[0], np.asarray(breaks, dtype=np.int64) + 1]))
    starts = starts[starts < n]
    ends = np.append(starts[1:], n)
    lens = ends - starts
    sigs = np.zeros((n, scheme.sig_len), dtype=np.uint8)
    heads = np.zeros((len(starts), 96), dtype=np.uint8)
    head_len = np.full(len(starts), 96, dtype=np.uint32)
    heads[0, :len(genesis_seed)] = np.frombuffer(genesis_seed, np.uint8)
    head_len[0] = len(genesis_seed)
    heads[1:] = rng.integers(0, 256, (len(starts) - 1, 96), dtype=np.uint8)
    rounds = np.arange(first_round, first_round + n, dtype=np.uint64)
    steps = int(lens.max())
    for p in range(steps):
        live = np.flatnonzero(lens > p)
        idx = starts[live] + p
        if p == 0:
            prev, plen = heads[live], head_len[live]
        else:
            prev, plen = sigs[idx - 1], np.full(len(idx), 96, dtype=np.uint32)
        sigs[idx] = scheme.sign_beacons(sk, rounds[idx], np.ascontiguousarray(prev), previous_lengths=plen)
        if progress and p % 512 == 0:
            progress(p, steps)
    return sigs


def corrupt(sigs, bad, rng):
    """Apply the three Cfg5 classes round-robin to rows `bad` (in place): (i) sigma + g2, (ii) one bit flipped,
    (iii) an on-curve point outside the subgroup. Returns the class of each corrupted row."""
    classes = []
    for k, i in enumerate(bad):
        c = k % 3
        if c == 0:
            sigs[i] = np.frombuffer(g2_synth.plus_generator(sigs[i].tobytes()), np.uint8)
        elif c == 1:
            sigs[i] = np.frombuffer(g2_synth.flip_bit(sigs[i].tobytes(), rng), np.uint8)
        else:
            sigs[i] = np.frombuffer(g2_synth.off_subgroup(rng), np.uint8)
        classes.append(c)
    return classes


def expected_faulty(bad, n):
    """The replay's faulty set: every corrupted round k and its successor k+1 (0-based, < n)."""
    s = set(int(k) for k in bad) | set(int(k) + 1 for k in bad if int(k) + 1 < n)
    return np.array(sorted(s), dtype=np.int64)


def stored_prevs(sigs, genesis_seed):
    """The previous-signature column a trimmed store yields: row 0 = genesis seed, row i = stored sigma_{i-1}."""
    n = len(sigs)
    prev = np.zeros((n, 96), dtype=np.uint8)
    prev[1:] = sigs[:-1]
    lens = np.full(n, 96, dtype=np.uint32)
    prev[0, :len(genesis_seed)] = np.frombuffer(genesis_seed, np.uint8)
    lens[0] = len(genesis_seed)
    return prev, lens
