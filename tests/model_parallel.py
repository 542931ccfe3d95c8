"""Design model (test infrastructure, pure Python, small cases only) of the PARALLEL
formulation the HIP kernels implement for referenceAssembler.build + all_contigs
(src/referenceassembler/referenceAssembler.py:25-111).

It exists to prove, on CPU and against the golden fixtures, that the data-parallel
restatement used on the GPU -- canonical counting with first-occurrence events,
oriented unitig links, path/cycle ranking, component start = first dict entry,
closed-form walk emulation -- gives exactly the reference's ordered contigs + links.
The kernels in pycuda-euler_amd/csrc/ follow this model step for step.
"""

COMP = {"A": "T", "C": "G", "G": "C", "T": "A"}


def twin(s):
    return "".join(COMP[c] for c in reversed(s))


def model_count(reads, k, read_base=0):
    """canonical key -> dict count contribution, string -> first insertion event"""
    cnt, first = {}, {}
    for r0, read in enumerate(reads):
        r = r0 + read_base
        wb = 0  # windows in earlier segments of this read
        for seg in read.split("N"):
            m = len(seg) - k + 1
            if m <= 0:
                continue
            for i in range(m):
                x = seg[i:i + k]
                t = twin(x)
                c = min(x, t)
                ef = (r << 32) | (2 * wb + i)               # forward insertion event
                er = (r << 32) | (2 * wb + 2 * m - 1 - i)   # twin(seg) insertion event
                cnt[c] = cnt.get(c, 0) + (2 if x == t else 1)
                first[x] = min(first.get(x, 1 << 62), ef)
                first[t] = min(first.get(t, 1 << 62), er)
            wb += m
    return cnt, first


def model_assemble(reads, k, limit=1):
    cnt, first = model_count(reads, k)
    solid = {c for c, v in cnt.items() if v > limit}
    return model_graph({c: cnt[c] for c in solid}, first, k)


def model_graph(cnt, first, k):
    """all_contigs from a solid set: cnt = canonical -> count, first = string -> first event"""
    solid = set(cnt)
    ind = lambda s: min(s, twin(s)) in solid  # noqa: E731
    fw = lambda s: [s[1:] + b for b in "ACGT"]  # noqa: E731
    bw = lambda s: [b + s[:-1] for b in "ACGT"]  # noqa: E731
    nodes = set()
    for c in solid:
        nodes.add(c)
        nodes.add(twin(c))
    # --- links ---------------------------------------------------------------------------
    succ, pred = {}, {}
    for x in nodes:
        f = [y for y in fw(x) if ind(y)]
        if len(f) == 1:
            y = f[0]
            if sum(ind(z) for z in bw(y)) == 1 and y != twin(x):
                succ[x] = y
                pred[y] = x
    # --- rank paths / cycles ---------------------------------------------------------------
    head, rank, cyc, plen = {}, {}, {}, {}
    for x in nodes:
        h, d, seen = x, 0, {x}
        while h in pred:
            h = pred[h]
            d += 1
            if h == x:
                break
        if h == x and x in pred:  # cycle
            cyc[x] = True
            # representative = min node; rank relative to it going forward
            ring = [x]
            y = succ[x]
            while y != x:
                ring.append(y)
                y = succ[y]
            rep = min(ring)
            j = ring.index(rep)
            head[x] = rep
            rank[x] = (len(ring) - j) % len(ring)
            plen[x] = len(ring)
        else:
            cyc[x] = False
            head[x] = h
            rank[x] = d
            t, n = x, d
            while t in succ:
                t = succ[t]
                n += 1
            plen[x] = n + 1
    # --- component min + start ------------------------------------------------------------
    pmin = {}
    for x in nodes:
        pmin[head[x]] = min(pmin.get(head[x], 1 << 62), first[x])
    starts = []
    for x in nodes:
        cm = min(pmin[head[x]], pmin[head[twin(x)]])
        if first[x] == cm:
            starts.append(x)
    starts.sort(key=lambda s: first[s])
    contigs = []
    for s in starts:
        n = plen[s]
        selftwin = head[twin(s)] == head[s]
        if not cyc[s]:
            if not selftwin:
                seq = [s]
                y = s
                while y in pred:
                    y = pred[y]
                    seq.insert(0, y)
                y = s
                while y in succ:
                    y = succ[y]
                    seq.append(y)
            else:
                p = [head[s]]
                while p[-1] in succ:
                    p.append(succ[p[-1]])
                nn = len(p) - 1
                j = rank[s]
                if 2 * j < nn:
                    seq = p[0:nn - j]
                elif 2 * j > nn:
                    seq = p[nn - j + 1:nn + 1]
                else:
                    seq = p
        else:
            ring = [s]
            while succ[ring[-1]] != s:
                ring.append(succ[ring[-1]])
            if not selftwin:
                seq = ring
            else:
                m = ring.index(twin(s))
                seq = ring if m == 0 else ring[m + 1:] + ring[:m]
        contigs.append(seq[0] + "".join(y[-1] for y in seq[1:]))
    # --- GFA links (all_contigs:90-109) ---------------------------------------------------
    heads, tails = {}, {}
    for i, x in enumerate(contigs):
        heads[x[:k]] = (i, "+")
        tails[twin(x[-k:])] = (i, "-")
    links = []
    for x in contigs:
        a, b = [], []
        for y in fw(x[-k:]):
            if y in heads:
                a.append(list(heads[y]))
            if y in tails:
                a.append(list(tails[y]))
        for z in fw(twin(x[:k])):
            if z in heads:
                b.append(list(heads[z]))
            if z in tails:
                b.append(list(tails[z]))
        links.append([a, b])
    order = sorted(((first[c], c) for c in solid))
    d = []
    for c in solid:
        for x in {c, twin(c)}:
            d.append((first[x], x, cnt[c]))
    d.sort()
    return [[x, v] for _, x, v in d], contigs, links
