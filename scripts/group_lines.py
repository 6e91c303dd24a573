"""Line model of k_cooc_group's reads at C4 1x1.

The heavy-row build (k_cooc_group, u16 rows = heavy rows under 65,536
listeners) reads, per index row s2: its listener ids (trs_users, 4 B each,
contiguous), every listener's record (urec: 16 u32 words = 64 B, one line),
and every listener's shard row part of each tile group (sr_songs, user-major,
shard-local ids, 16-B chunks from the part's first entry, the last chunk
over-reading up to 3 entries). This script replays mr_load's row
classification and layout on the CPU (renumbered users by degree, the tile
groups of 4 x 19,456 songs) and counts 128-B lines per array:

  upper  every line fetched per use: per (row, group) for the big rows (one
         workgroup per (row, group)), per group walk for the pipelined rows
  lower  every line once per row (perfect L2 reuse inside a row)

against the byte model (4 B per listener id and per shard-row entry, once).
Compare with the kernel's measured fetch (rocprofv3 FETCH_SIZE x 2,
profiles/r04/s45/pmc_c4_kernels.txt: 28.46 GB per C4 step).

usage: python scripts/group_lines.py [--out FILE]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from musicrecommendation_amd import synth  # noqa: E402

BS, NT, GRP = 19456, 20, 4          # C4 1x1: tiles of 19,456 songs, 4 tiles per k_cooc_group pass
NG = (NT + GRP - 1) // GRP
BIG_ROW, U32_ROW = 2048, 65536       # kCoocBigRow, u32-counter rows
LIGHT_SLOTS, LIGHT_LOAD, LIGHT_CNT = 32768, 80, 4095
LINE = 128


def span_lines(a, e):
    """Lines touched by byte range [4a, 4e) (e > a), vectorised."""
    return ((4 * (e - 1)) >> 7) - ((4 * a) >> 7) + 1


def main():
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    t0 = time.time()
    ds = synth.config("c4").dataset()
    n_tr, n_s = ds.n_train, ds.n_songs
    deg = np.diff(ds.tr_off).astype(np.int64)
    perm = np.argsort(-deg, kind="stable")            # new id -> old id
    inv = np.empty(n_tr, np.int64)
    inv[perm] = np.arange(n_tr)
    deg_new = deg[perm]
    p_off = np.zeros(n_tr + 1, np.int64)
    np.cumsum(deg_new, out=p_off[1:])
    user_old = np.repeat(np.arange(n_tr, dtype=np.int64), deg)
    songs = ds.tr_songs.astype(np.int64)
    # per user: its first entry of every tile (the urec starts), new ids
    cnt = np.bincount(user_old * NT + songs // BS, minlength=n_tr * NT).reshape(n_tr, NT)
    st = np.zeros((n_tr, NT + 1), np.int64)
    np.cumsum(cnt, axis=1, out=st[:, 1:])
    st = st[perm]
    del cnt
    # song -> listeners (new ids, ascending)
    newu = inv[user_old]
    del user_old
    order = np.lexsort((newu, songs))
    trs_users = newu[order]
    del order, newu
    c_tr = np.bincount(songs, minlength=n_s).astype(np.int64)
    trs_off = np.zeros(n_s + 1, np.int64)
    np.cumsum(c_tr, out=trs_off[1:])
    # index rows: distinct test-visible songs with train listeners, heaviest first
    rs = np.unique(ds.te_songs)
    rs = rs[c_tr[rs] > 0]
    rs = rs[np.lexsort((rs, -c_tr[rs]))]
    # entry bound of each row: Σ_{v ∈ L(s2)} deg(v)
    bound_all = np.add.reduceat(deg_new[trs_users], trs_off[:-1].clip(max=len(trs_users) - 1))
    bound = np.where(c_tr[rs] > 0, bound_all[rs], 0)
    light = (np.minimum(bound, n_s) * 100 <= LIGHT_SLOTS * LIGHT_LOAD) & (c_tr[rs] <= LIGHT_CNT)
    heavy = rs[~light]
    h16 = heavy[c_tr[heavy] < U32_ROW]
    big = c_tr[h16] >= BIG_ROW
    res = {"rows": int(rs.size), "light_rows": int(light.sum()), "heavy_rows": int(heavy.size),
           "u32_rows": int((c_tr[heavy] >= U32_ROW).sum()), "u16_rows": int(h16.size),
           "big_rows": int(big.sum()), "pipelined_rows": int((~big).sum())}
    # per (row, listener) over the u16 heavy rows
    parts = {k: 0 for k in ("ids_bytes", "rows_bytes", "ids_lines_lower", "ids_lines_upper", "urec_lines_lower",
                            "urec_lines_upper", "sr_lines_lower", "sr_lines_upper", "sr_lines_per_group_walk",
                            "sr_lines_upper_aligned", "lrec_lines_upper")}
    hist = {}
    for is_big in (True, False):
        rows = h16[big] if is_big else h16[~big]
        if rows.size == 0:
            continue
        # listener ids: contiguous per row
        a, n = trs_off[rows], c_tr[rows]
        idl = span_lines(a, a + n)
        parts["ids_bytes"] += int(4 * n.sum())
        parts["ids_lines_lower"] += int(idl.sum())
        parts["ids_lines_upper"] += int(idl.sum() * (NG if is_big else 1))
        # listeners of these rows, in chunks (memory)
        for c0 in range(0, rows.size, 2000):
            rr = rows[c0:c0 + 2000]
            lst = np.concatenate([trs_users[trs_off[s]:trs_off[s + 1]] for s in rr])
            parts["rows_bytes"] += int(4 * deg_new[lst].sum())
            # urec records: 64 B each, one line per fetch
            parts["urec_lines_lower"] += int(lst.size)
            parts["urec_lines_upper"] += int(lst.size * (NG if is_big else 1))
            base = p_off[lst]
            lo_all = base + st[lst, 0]
            hi_all = base + st[lst, NT]
            nz = hi_all > lo_all
            parts["sr_lines_lower"] += int(span_lines(lo_all[nz], hi_all[nz] + 3).sum())
            tot = np.zeros(lst.size, np.int64)
            tal = np.zeros(lst.size, np.int64)
            for g in range(NG):
                aa = base + st[lst, g * GRP]
                bb = base + st[lst, min(NT, (g + 1) * GRP)]
                m = bb > aa
                last = aa + 4 * ((bb - 1 - aa) // 4) + 3  # the last 16-B chunk's last entry
                tot[m] += span_lines(aa[m], last[m] + 1)
                tal[m] += span_lines(aa[m], bb[m])  # 16-B-aligned chunks: the lines of [a, b) only
            parts["sr_lines_upper"] += int(tot.sum())
            parts["sr_lines_upper_aligned"] += int(tal.sum())
            # per-(row, listener) 16-B records (lrec), contiguous: per row, per group for big rows
            parts["lrec_lines_upper"] += int(np.ceil(16 * lst.size / LINE) * (NG if is_big else 1))
            parts["sr_lines_per_group_walk"] += int(tot.sum())
        ct = c_tr[rows]
        for lo_, hi_ in ((0, 256), (256, 1024), (1024, 2048), (2048, 8192), (8192, 65536)):
            m = (ct >= lo_) & (ct < hi_)
            key = f"c_tr [{lo_}, {hi_})"
            h = hist.setdefault(key, {"rows": 0, "listeners": 0})
            h["rows"] += int(m.sum())
            h["listeners"] += int(ct[m].sum())
    GB = 1e9
    res["algorithmic_GB"] = {"listener_ids": parts["ids_bytes"] / GB, "shard_rows": parts["rows_bytes"] / GB}
    res["line_model_GB"] = {
        "listener_ids": [parts["ids_lines_lower"] * LINE / GB, parts["ids_lines_upper"] * LINE / GB],
        "urec_records": [parts["urec_lines_lower"] * LINE / GB, parts["urec_lines_upper"] * LINE / GB],
        "shard_row_chunks": [parts["sr_lines_lower"] * LINE / GB, parts["sr_lines_upper"] * LINE / GB],
    }
    res["shard_row_chunks_aligned_upper_GB"] = parts["sr_lines_upper_aligned"] * LINE / GB
    res["lrec_records_upper_GB"] = parts["lrec_lines_upper"] * LINE / GB
    lo = sum(v[0] for v in res["line_model_GB"].values())
    hi = sum(v[1] for v in res["line_model_GB"].values())
    res["line_model_total_GB"] = [lo, hi]
    res["heavy_u16_rows_by_listeners"] = hist
    res["seconds"] = time.time() - t0
    res["note"] = ("[lower, upper]: lines once per row vs once per use (big rows: per (row, group) workgroup; "
                   "pipelined rows: per group walk for the shard-row chunks); 128-B lines")
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
