"""Loading the committed golden fixtures (tests/golden/, made by tools/make_golden.py)."""
import json
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INDEX = {"tiny": os.path.join(GOLD, "index", "tiny.fa"), "rep": os.path.join(GOLD, "index", "rep.fa"),
         "nrun": os.path.join(GOLD, "index", "nrun.fa")}


def cases():
    with open(os.path.join(GOLD, "manifest_tiny.json")) as f:
        return json.load(f)


def limits_cases():
    """Cases past the fast search kernel's layouts (tools/make_golden.py --limits)."""
    with open(os.path.join(GOLD, "manifest_limits.json")) as f:
        return json.load(f)


def load_case(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["args"] = str(d["args"]).split()
    d["index"] = str(d["index"])
    d["batch"] = int(d["batch"])
    return d


def split_hits(n_aln, hits):
    """Per-read list of (n_aln, 9) uint32 arrays."""
    out, o = [], 0
    for na in n_aln:
        na = max(int(na), 0)
        out.append(hits[o:o + na])
        o += na
    return out


def parse_opts(args, base):
    """Apply `HSA aln`-style flags (bwtaln.c:539-575) to an option dict."""
    o = dict(base)
    i = 0
    opte = -1
    while i < len(args):
        a = args[i]
        v = args[i + 1] if i + 1 < len(args) else "0"
        if a == "-n":
            if "." in v:
                o["fnr"], o["max_diff"] = float(v), -1
            else:
                o["max_diff"], o["fnr"] = int(v), -1.0
            i += 1
        elif a in ("-o", "-M", "-O", "-E", "-d", "-i", "-l", "-k", "-m", "-R", "-B", "-e"):
            key = {"-o": "max_gapo", "-M": "s_mm", "-O": "s_gapo", "-E": "s_gape", "-d": "max_del_occ",
                   "-i": "indel_end_skip", "-l": "seed_len", "-k": "max_seed_diff", "-m": "max_entries",
                   "-R": "max_top2", "-B": None, "-e": "opte"}[a]
            if key == "opte":
                opte = int(v)
            elif key:
                o[key] = int(v)
            i += 1
        elif a == "-L":
            o["mode"] |= 0x04
        elif a == "-N":
            o["mode"] |= 0x10
            o["max_top2"] = 0x7FFFFFFF
        i += 1
    if opte > 0:
        o["max_gape"] = opte
        o["mode"] &= ~0x01
    return o


def main_path_digest(n_aln, flags, hits):
    """Same definition as tools/make_golden.py hits_digest()."""
    import hashlib
    h = hashlib.sha256()
    splice = (np.asarray(flags) & 1).astype(bool)
    na = np.where(splice, -1, np.asarray(n_aln, np.int32)).astype(np.int32)
    h.update(na.tobytes())
    keep = np.repeat(~splice, np.maximum(np.asarray(n_aln, np.int64), 0))
    h.update(np.ascontiguousarray(np.asarray(hits, np.uint32)[keep], np.uint32).tobytes())
    return h.hexdigest()


MGCAP_CASES = ["mgcap_default", "mgcap_n4o1"]


def load_mgcap(name):
    """bwt_match_gap calls recorded from the reference (tools/make_golden.py --mgcap):
    per call strand, len, seed kind (0 NULL, 1 own, 2 aliased), n_stacks, the option
    block, the searched sequence, widths before/after and the hits."""
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    hdr, opt = z["hdr"], z["opt"]
    L = hdr[:, 1].astype(np.int64)
    so = np.concatenate([[0], np.cumsum(L)])
    wo = np.concatenate([[0], np.cumsum(L + 1)])
    sd = np.concatenate([[0], np.cumsum(hdr[:, 4].astype(np.int64))])
    ho = np.concatenate([[0], np.cumsum(np.maximum(z["n_aln"], 0).astype(np.int64))])
    calls = []
    for j in range(len(hdr)):
        calls.append(dict(strand=int(hdr[j, 0]), len=int(L[j]), seed=int(hdr[j, 2]), n_stacks=int(hdr[j, 3]),
                          opt=opt[j].copy(), seq=z["seq"][so[j]:so[j + 1]],
                          wb=z["wb"][wo[j]:wo[j + 1]], ws=z["ws"][sd[j]:sd[j + 1]],
                          hits=z["hits"][ho[j]:ho[j + 1]], wo=z["wo"][wo[j]:wo[j + 1]]))
    return calls


def ecoli_manifest():
    with open(os.path.join(GOLD, "manifest_ecoli.json")) as f:
        return json.load(f)


EXTCAP_CASES = ["extcap_default", "extcap_n4o1"]


def load_extcap(name):
    """Seed extensions recorded from the reference (tools/make_golden.py --extcap): per
    call the header (dir, len, strand, n_stacks, max_pos in, window lo, window n, read
    length), the option block, aln in/out, the window of sequence and width bids, and
    (ret, max_pos out).  Yields dicts."""
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    hdr, opt, ai, ao, tail = z["hdr"], z["opt"], z["aln_in"], z["aln_out"], z["tail"]
    seq, bid = z["seq"], z["bid"]
    off = np.concatenate([[0], np.cumsum(hdr[:, 6].astype(np.int64))])
    for j in range(len(hdr)):
        yield dict(dir=int(hdr[j, 0]), len=int(hdr[j, 1]), strand=int(hdr[j, 2]), n_stacks=int(hdr[j, 3]),
                   max_pos=int(hdr[j, 4]), lo=int(hdr[j, 5]), read_len=int(hdr[j, 7]), opt=opt[j],
                   aln_in=ai[j], aln_out=ao[j], ret=int(tail[j, 0]), max_pos_out=int(tail[j, 1]),
                   seq=seq[off[j]:off[j + 1]], bid=bid[off[j]:off[j + 1]])
