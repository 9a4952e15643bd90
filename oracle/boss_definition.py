"""TEST INFRASTRUCTURE ONLY -- a second, independent restatement of the BOSS table.

Where oracle/boss_oracle.c follows the reference's streaming code line by line, this module
builds the same table from the *definition* of a BOSS graph over strings, for small inputs:

* real edges  = every (k+1)-window over {A,C,G,T} (U -> T, case-insensitive) of each sequence,
  plus reverse complements in canonical mode (boss_chunk_construct.cpp:179-222);
* dummy sink  = node v + '$' for every edge target node v with no real out-edge (:54-98);
* dummy source= for every real source node u without a real in-edge, the edges
  '$'^j + u[:k-j] -> u[k-j] for j = 1..k (:123-168, :286-306), plus the root '$'^k -> '$';
* rows sorted co-lexicographically by node (last char most significant), then by label;
* last / W (+5 'minus' for a repeated label among nodes sharing node[1:]) / F / weights as
  initialize_chunk (boss_chunk.cpp:32-133) defines them, with the leading row 0.

It shares no code with the C restatement, so agreement of the two pins the bit-level rules
(packing, rc, lift, iterator joins) against plain string semantics.
"""

ALPH = "$ACGT"
CODE = {c: i for i, c in enumerate(ALPH)}
COMP = {"A": "T", "C": "G", "G": "C", "T": "A"}


def _norm(seq):
    out = []
    for ch in seq:
        u = ch.upper()
        if u == "U":
            u = "T"
        out.append(u if u in "ACGT" else None)
    return out


def revcomp(s):
    return "".join(COMP[c] for c in reversed(s))


def real_edges(k, seqs, canonical=False, counts=None, cmax=None):
    K = k + 1
    cnt = {}
    for idx, seq in enumerate(seqs):
        c = 1 if counts is None else int(counts[idx])
        if cmax is not None:
            c = min(c, cmax)
        s = _norm(seq)
        for i in range(0, len(s) - K + 1):
            w = s[i:i + K]
            if any(x is None for x in w):
                continue
            e = "".join(w)
            cnt[e] = cnt.get(e, 0) + c
            if canonical:
                r = revcomp(e)
                cnt[r] = cnt.get(r, 0) + c
    if cmax is not None:
        cnt = {e: min(v, cmax) for e, v in cnt.items()}
    return cnt


def boss_table(k, seqs, canonical=False, bits_per_count=0, counts=None):
    cmax = None
    if bits_per_count:
        cmax = 255 if bits_per_count <= 8 else 65535 if bits_per_count <= 16 else 2**32 - 1
    edges = real_edges(k, seqs, canonical, counts, cmax)
    out_nodes = {e[:k] for e in edges}
    in_keys = {(e[1:k], e[k]) for e in edges}  # (source node minus first char, label)
    rows = dict((e, c) for e, c in edges.items())
    for e in edges:
        v = e[1:]
        if v not in out_nodes:
            rows[v + "$"] = 0
    for e in edges:
        u = e[:k]
        if (u[:k - 1], u[k - 1]) in in_keys:
            continue
        for j in range(1, k + 1):
            rows["$" * j + u[:k - j] + u[k - j]] = 0
    rows["$" * (k + 1)] = 0

    def key(s):
        return (tuple(CODE[c] for c in reversed(s[:k])), CODE[s[k]])

    order = sorted(rows, key=key)
    W, last, weights = [0], [0], [0]
    F = [0] * 5
    seen = {}
    wmax = (1 << bits_per_count) - 1 if bits_per_count else 0
    for i, s in enumerate(order):
        node, label = s[:k], CODE[s[k]]
        last.append(1 if i + 1 == len(order) or order[i + 1][:k] != node else 0)
        w = label
        if label:
            g = (node[1:], label)
            if g in seen:
                w = label + 5
            seen[g] = True
        W.append(w)
        c = rows[s]
        weights.append(min(c, wmax) if (c and label and node[0] != "$") else 0)
    tops = [CODE[s[k - 1]] for s in order]
    for c in range(1, 5):
        F[c] = sum(1 for t in tops if t < c)
    return {"W": W, "last": last, "F": F, "weights": weights if bits_per_count else None,
            "n_real": len(edges), "rows": order}
