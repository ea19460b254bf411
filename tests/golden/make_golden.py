#!/usr/bin/env python3
"""Golden-vector generator: a brute-force, definition-level restatement of ntcomp's
encode/decode hot path.  TEST INFRASTRUCTURE ONLY -- never imported by the product.

Parity status: UNPINNED against the real reference.  The reference (tmaklin/ntcomp,
Rust) and the crates holding its index semantics (sbwt 0.3.11, kbo 0.5.1, bitnuc
0.2.11; Cargo.lock:1358-1361, 740-743, 145-148) are not buildable in this image (no
Rust toolchain, no crate sources, no network), and the reference's own test
(tests/fasta_data.rs:28-101) pins only the round-trip property.  This script restates
the published algorithms from first principles, deliberately WITHOUT any rank/select or
streaming machinery, so that it is an independent check on oracle/ntcomp_oracle.c (the
faithful restatement) and on the HIP kernels:

  * SBWT node set (Alanko et al. SBWT; sbwt 0.3.11 as driven by kbo::build with
    add_revcomp=true, main.rs:118): the k-spectrum plus, for every k-mer without an
    in-neighbour, the dummy nodes $^(k-i) x[0..i] for i=0..k-1 (i=0 is the root $^k,
    which is always present).  Nodes sorted colexicographically, '$' < A < C < G < T.
  * subset label of node v: {c : v[1:]+c is a node}, kept only on the colex-first node
    of each (k-1)-suffix group.  C[c] = 1 + #labels with a character < c.
  * LCS[i] = longest common suffix of nodes i-1 and i; LCS[0] = 0.
  * matching statistics (StreamingIndex::matching_statistics, lib.rs:172-173) BY
    DEFINITION: d_p = longest suffix (<= k) of q[0..p] that is a suffix of some node;
    start = first node (colex) having that suffix (start 0 when d = 0).
  * encode_sequence (lib.rs:163-230) transcribed loop for loop, with left_extend_kmer
    (lib.rs:94-128) doing its 4 x search() per step where search(kmer) is k-mer set
    membership.
  * encode_dictionary (encode.rs:129-166) record words; bitnuc as_2bit = LSB-first
    A=0,C=1,G=2,T=3 ([ext, recalled] bitnuc 0.2.11).
  * decode_sequence (lib.rs:254-318) with access_kmer = the node string and
    left_extend_kmer2 (lib.rs:130-161).

Usage: python tests/golden/make_golden.py   (rewrites tests/golden/*.json.gz)
"""
import bisect
import gzip
import json
import os
import random

ALPHA = "ACGT"
COMP = {"A": "T", "C": "G", "G": "C", "T": "A"}
HERE = os.path.dirname(os.path.abspath(__file__))


def revcomp(s):
    return "".join(COMP[c] for c in reversed(s))


def kmer_spectrum(seqs, k, add_revcomp=True):
    """k-mers of every maximal ACGT run (kbo/sbwt skip k-mers with other bytes)."""
    out = set()
    for s in seqs:
        s = s.upper()
        runs, cur = [], []
        for ch in s:
            if ch in COMP:
                cur.append(ch)
            else:
                if cur:
                    runs.append("".join(cur))
                cur = []
        if cur:
            runs.append("".join(cur))
        for r in runs:
            for i in range(len(r) - k + 1):
                x = r[i:i + k]
                out.add(x)
                if add_revcomp:
                    out.add(revcomp(x))
    return out


class NaiveSBWT:
    def __init__(self, seqs, k, add_revcomp=True):
        self.k = k
        K = kmer_spectrum(seqs, k, add_revcomp)
        self.kmers = K
        nodes = set(K)
        for x in K:
            pre = x[:-1]
            if not any(c + pre in K for c in ALPHA):
                for i in range(k):
                    nodes.add("$" * (k - i) + x[:i])
        nodes.add("$" * k)
        self.order = sorted(nodes, key=lambda s: s[::-1])
        self.rev = [s[::-1] for s in self.order]
        self.n = len(self.order)
        nodeset = nodes
        self.sets = []
        for i, v in enumerate(self.order):
            if i > 0 and self.order[i - 1][1:] == v[1:]:
                self.sets.append("")
            else:
                self.sets.append("".join(c for c in ALPHA if v[1:] + c in nodeset))
        self.lcs = [0] * self.n
        for i in range(1, self.n):
            a, b = self.order[i - 1], self.order[i]
            t = 0
            while t < k and a[k - 1 - t] == b[k - 1 - t]:
                t += 1
            self.lcs[i] = t
        cnt = [sum(1 for s in self.sets if c in s) for c in ALPHA]
        self.C = [1 + sum(cnt[:j]) for j in range(4)]

    # --- queries by definition -------------------------------------------------------
    def suffix_range(self, alpha):
        """colex interval of nodes whose suffix is alpha (alpha has no '$')."""
        ra = alpha[::-1]
        lo = bisect.bisect_left(self.rev, ra)
        hi = lo
        while hi < self.n and self.rev[hi].startswith(ra):
            hi += 1
        return lo, hi

    def search(self, pattern):
        lo, hi = self.suffix_range(pattern)
        return (lo, hi) if hi > lo else None

    def access_kmer(self, j):
        return self.order[j]

    def matching_statistics(self, q):
        res = []
        d = 0
        for p in range(1, len(q) + 1):
            t = min(self.k, d + 1, p)
            while t > 0:
                lo, hi = self.suffix_range(q[p - t:p])
                if hi > lo:
                    break
                t -= 1
            if t == 0:
                res.append((0, 0))
            else:
                res.append((t, self.suffix_range(q[p - t:p])[0]))
            d = t
        return res

    def rows_bytes(self):
        words = (self.n + 63) // 64
        out = {}
        for c in ALPHA:
            bits = bytearray(words * 8)
            for j, s in enumerate(self.sets):
                if c in s:
                    bits[j // 8] |= 1 << (j % 8)
            out[c] = bits.hex()
        return out


# --- lib.rs:94-128 ------------------------------------------------------------------
def left_extend_kmer(kmer_start, ref_nts, sb, max_ext):
    ext = 0
    kmer = kmer_start
    while ext < max_ext:
        hits = []
        for c in ALPHA:
            nk = c + kmer[0:len(kmer) - (ext + 1)]
            r = sb.search(nk)
            if r is not None:
                hits.append((nk, r))
        if hits:
            seq_matches = hits[0][0][0] == ref_nts[len(ref_nts) - len(kmer) - 1]
            if seq_matches and len(hits) == 1 and hits[0][1][1] - hits[0][1][0] == 1:
                kmer = hits[0][0][0] + kmer
            else:
                break
        else:
            break
        ext += 1
    return kmer


# --- lib.rs:130-161 ------------------------------------------------------------------
def left_extend_kmer2(kmer_start, sb, max_ext):
    ext = 0
    kmer = kmer_start
    while ext < max_ext:
        hits = []
        for c in ALPHA:
            nk = c + kmer[0:len(kmer) - (ext + 1)]
            r = sb.search(nk)
            if r is not None:
                hits.append((nk, r))
        if hits and len(hits) == 1 and hits[0][1][1] - hits[0][1][0] == 1:
            kmer = hits[0][0][0] + kmer
        else:
            break
        ext += 1
    return kmer


# --- lib.rs:163-230 ------------------------------------------------------------------
def encode_sequence(q, sb):
    k = sb.k
    n = len(q)
    if n == 0:
        raise ValueError("EncodeError")
    res = [list(x) for x in sb.matching_statistics(q)]
    if any(d == 0 for d, _ in res):
        raise ValueError("base absent from index: the reference never terminates (lib.rs:207)")
    i = n
    kept = []
    while i > 0:
        st = res[i - 1][1]
        if res[i - 1][0] == k and i > k + 1:
            kmer = sb.access_kmer(st)
            assert kmer == q[i - len(kmer):i]
            new_kmer = left_extend_kmer(kmer, q[0:i], sb, i - k - 1)
            match_len = len(new_kmer)
            old_i = i
            while True:
                if res[i - 1][0] < match_len:
                    old_ms = res[i - 1][0]
                    i -= old_ms
                    match_len -= old_ms
                else:
                    res[old_i - 1][0] = len(new_kmer) - (match_len - 1)
                    kept.append(old_i - 1)
                    break
        else:
            kept.append(i - 1)
            if i > res[i - 1][0]:
                i -= res[i - 1][0] - 1
            else:
                break
        if i > 0:
            i -= 1
        else:
            break
    dic = [(res[x][0], res[x][1], x + 1) for x in kept]  # (len, colex start, end)
    assert max(d for d, _, _ in dic) < (1 << 24)
    assert sum(d for d, _, _ in dic) == n
    return dic


def as_2bit(seq):
    v = 0
    for j, ch in enumerate(seq):
        v |= ALPHA.index(ch) << (2 * j)
    return v


def from_2bit(v, length):
    return "".join(ALPHA[(v >> (2 * j)) & 3] for j in range(length))


# --- encode.rs:129-166 ---------------------------------------------------------------
def encode_dictionary(dic, sb):
    k = sb.k
    out = []
    first = True
    for length, start, _end in dic:
        if length > 11:
            w = (start & 0xFFFFFFFF) | ((length & 0xFFFFFF) << 32) | (int(first) << 56)
        else:
            kmer = sb.access_kmer(start)
            seq = kmer[k - length:k]
            w = (as_2bit(seq) & ((1 << 56) - 1)) | (((int(first) + 2) | (length << 2)) << 56)
        out.append(w)
        first = False
    return out


# --- lib.rs:254-318 ------------------------------------------------------------------
def decode_sequence(encoding, sb):
    k = sb.k
    seqs, seq = [], []
    for rec in reversed(encoding):
        flag = (rec >> 56) & 0xFF
        first = flag & 1
        if flag & 2 == 0:
            colex = rec & 0xFFFFFFFF
            slen = (rec >> 32) & 0xFFFFFF
            if slen > k:
                kmer = left_extend_kmer2(sb.access_kmer(colex), sb, slen - k)
                assert len(kmer) == slen
            else:
                kmer = sb.access_kmer(colex)
            seq.append(kmer[len(kmer) - slen:])
        else:
            seq.append(from_2bit(rec & ((1 << 56) - 1), flag >> 2))
        if first:
            seqs.append("".join(seq))
            seq = []
    return list(reversed(seqs))


def rand_seq(rng, n):
    return "".join(rng.choice(ALPHA) for _ in range(n))


def mutate(rng, s, rate):
    out = list(s)
    for j in range(len(out)):
        if rng.random() < rate:
            out[j] = rng.choice([c for c in ALPHA if c != out[j]])
    return "".join(out)


def make_reads(rng, seqs, k, n_reads, read_len, err):
    reads = []
    genome = [s for s in seqs if len(s) >= read_len]
    for r in range(n_reads):
        g = rng.choice(genome)
        st = rng.randrange(0, len(g) - read_len + 1)
        x = g[st:st + read_len]
        if rng.random() < 0.5:
            x = revcomp(x)
        reads.append(mutate(rng, x, err))
    # edge cases: lengths around k and the 11-base short-record threshold
    g = genome[0]
    for L in sorted({1, 2, 11, 12, k - 1, k, k + 1, k + 2, 2 * k + 3}):
        if 0 < L <= len(g):
            reads.append(g[5:5 + L] if 5 + L <= len(g) else g[:L])
    reads.append(rand_seq(rng, read_len))  # unrelated read: many short records
    reads.append(g[:read_len])  # starts at a source k-mer (dummy-rooted MS)
    reads.append(revcomp(g[-read_len:]))
    return reads


def case(name, seed, k, contig_lens, n_reads, read_len, err):
    rng = random.Random(seed)
    seqs = [rand_seq(rng, L) for L in contig_lens]
    sb = NaiveSBWT(seqs, k)
    reads = make_reads(rng, seqs, k, n_reads, read_len, err) if read_len else list(seqs)
    ms, recs = [], []
    for q in reads:
        ms.append(sb.matching_statistics(q))
        recs.append(encode_dictionary(encode_sequence(q, sb), sb))
    flat = [w for r in recs for w in r]
    assert decode_sequence(flat, sb) == reads
    obj = {
        "name": name, "seed": seed, "k": k, "add_revcomp": True, "seqs": seqs,
        "n": sb.n, "C": sb.C, "rows": sb.rows_bytes(), "lcs": bytes(sb.lcs).hex(),
        "reads": reads, "ms": ms, "records": recs,
    }
    path = os.path.join(HERE, name + ".json.gz")
    with gzip.open(path, "wt") as f:
        json.dump(obj, f, separators=(",", ":"))
    print(f"{name}: k={k} n={sb.n} reads={len(reads)} records={len(flat)} -> {path}")


def main():
    case("small_k15", 11, 15, [700, 300], 40, 60, 0.02)
    case("ecoli_like_k31", 12, 31, [3000], 60, 150, 0.01)
    case("k91_perfect", 13, 91, [2500], 30, 150, 0.0)
    case("k91_err", 14, 91, [2500], 40, 150, 0.01)
    # reference test shape (tests/fasta_data.rs:40-60): 7 random contigs < 2000 bp,
    # k = 255, the contigs themselves are the reads.  (random 0.14 is unavailable, so
    # the contigs come from our own seeded generator.)
    rng = random.Random(20250731)
    lens = [rng.randrange(0, 2000) for _ in range(7)]
    lens = [L if L > 0 else 1 for L in lens]
    case("fasta_data_k255", 20250731, 255, lens, 0, 0, 0.0)


if __name__ == "__main__":
    main()
