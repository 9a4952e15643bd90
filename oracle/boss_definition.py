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

    out = table_from_rows(k, rows, bits_per_count)
    out["n_real"] = len(edges)
    return out


def _key(k):
    return lambda s: (tuple(CODE[c] for c in reversed(s[:k])), CODE[s[k]])


def table_from_rows(k, rows, bits_per_count=0):
    """initialize_chunk (boss_chunk.cpp:32-133) over a set of (k+1)-mer strings -> counts: rows
    sorted co-lexicographically by node then label; a `$` label whose node does not end with `$`
    is skipped when the next row has the same node (a redundant dummy sink); last = the next row
    has another node; W + 5 when an earlier emitted row of the same node[1:] has the label."""
    order = sorted(rows, key=_key(k))
    W, last, weights = [0], [0], [0]
    F = [0] * 5
    seen = {}
    kept = []
    wmax = (1 << bits_per_count) - 1 if bits_per_count else 0
    for i, s in enumerate(order):
        node, label = s[:k], CODE[s[k]]
        same_next = i + 1 < len(order) and order[i + 1][:k] == node
        if same_next and label == 0 and node[-1] != "$":
            continue
        kept.append(s)
        last.append(0 if same_next else 1)
        w = label
        if label:
            g = (node[1:], label)
            if g in seen:
                w = label + 5
            seen[g] = True
        W.append(w)
        c = rows[s]
        weights.append(min(c, wmax) if (c and label and node[0] != "$") else 0)
    tops = [CODE[s[k - 1]] for s in kept]
    for c in range(1, 5):
        F[c] = sum(1 for t in tops if t < c)
    return {"W": W, "last": last, "F": F, "weights": weights if bits_per_count else None,
            "rows": kept}


def generate_suffixes(length):
    """KmerExtractorBOSS::generate_suffixes (kmer/kmer_extractor.cpp:402-416) over
    utils::generate_strings (common/utils/string_utils.cpp:82-95): every string over $ACGT of
    the length, the LAST char varying slowest, keeping those whose `$`s form a prefix."""
    out = [""]
    while len(out[0]) < length:
        head = out.pop(0)
        out.extend(c + head for c in ALPH)
    res = []
    for s in out:
        j = s.rfind("$")
        if j < 0 or s[:j + 1] == "$" * (j + 1):
            res.append(s)
    return res


def _segments(seq):
    s = _norm(seq)
    seg = []
    for x in s + [None]:
        if x is None:
            if seg:
                yield "".join(seg)
            seg = []
        else:
            seg.append(x)


def suffix_rows(k, seqs, suffix, both=False, counts=None, cmax=None):
    """The suffix-filtered collector by definition (kmer_extractor.cpp:316-381): each segment
    of valid chars of length >= k + 1, read as '$'*k + segment + '$', gives its (k+1)-windows;
    keep those whose node ends with `suffix`; BOTH mode also scans the reverse complement of
    every read; the all-'$' suffix adds '$'*(k+1)."""
    K = k + 1
    ns = len(suffix)
    rows = {}
    for idx, seq in enumerate(seqs):
        c = 1 if counts is None else int(counts[idx])
        if cmax is not None:
            c = min(c, cmax)
        strands = [seq]
        if both:
            comp = {"A": "T", "C": "G", "G": "C", "T": "A", "U": "A",
                    "a": "t", "c": "g", "g": "c", "t": "a", "u": "a"}
            strands.append("".join(comp.get(ch, "N") for ch in reversed(seq)))
        for st in strands:
            for seg in _segments(st):
                if len(seg) < K:
                    continue
                padded = "$" * k + seg + "$"
                for i in range(len(padded) - K + 1):
                    w = padded[i:i + K]
                    if w[K - 1 - ns:K - 1] == suffix:
                        rows[w] = rows.get(w, 0) + c
    if suffix and set(suffix) == {"$"}:
        rows["$" * K] = rows.get("$" * K, 0) + 1
    if cmax is not None:
        rows = {e: min(v, cmax) for e, v in rows.items()}
    return rows


def suffix_table(k, seqs, suffix, both=False, bits_per_count=0, counts=None):
    cmax = None
    if bits_per_count:
        cmax = 255 if bits_per_count <= 8 else 65535 if bits_per_count <= 16 else 2**32 - 1
    return table_from_rows(k, suffix_rows(k, seqs, suffix, both, counts, cmax), bits_per_count)


def prune_rows(k, rows):
    """erase_redundant_dummy_edges by definition (boss.cpp:1443-1650): a source-dummy edge
    ($-prefixed node) is kept iff some depth-k dummy edge below it ('$' + v -> b, below when
    v + b starts with the edge's non-'$' chars + label) enters a node v + b that has no other
    incoming edge.  Returns the kept row strings (the main dummy edge always stays)."""
    rows = list(rows)
    incoming = {}
    for r in rows:
        if r[k] != "$":
            tgt = r[1:k] + r[k]
            incoming[tgt] = incoming.get(tgt, 0) + 1
    ends = [r[1:k] + r[k] for r in rows
            if r[0] == "$" and "$" not in r[1:] and incoming.get(r[1:k] + r[k], 0) == 1]
    keep = []
    for r in rows:
        if r[0] != "$" or r == "$" * (k + 1):
            keep.append(r)
            continue
        p = r[:k].lstrip("$") + r[k]
        if any(e.startswith(p) for e in ends):
            keep.append(r)
    return keep
