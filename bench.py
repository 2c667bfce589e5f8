#!/usr/bin/env python3
"""bench.py -- embedding lookups/s on the DLRM Criteo-Terabyte shape.

One step = one pass of the north_star hot path over one batch: for each of
the 26 sparse features, EmbeddingVariable insert-on-miss resolve of every id
-> gather + sum pooling into the [B, 26*128] input_layer output
(embedding_lookup_sparse, combiner "sum", hotness 1; forward-only lookups of
filter-free EVs need no Unique), one fused kernel at N = 1.
At N GPUs the tables are row-sharded (owner = key % N) and every step sends
the ids to their owners, resolves them there and brings the rows back: over
xGMI peer writes (XgmiShardedLookup), or the RCCL all-to-all engine
(ShardedLookup) when IPC mapping is unavailable; per-GPU work is fixed
(weak scaling).  The JSON line carries the roofline of the dominant kernel
and, for the north_star's row-gather target, of the pre-resolved gather.

Timing: W untimed warmup steps, then exactly K steps bracketed by a barrier
and torch.cuda.synchronize(); max over ranks; rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))

# before HIP initialises: graph replays without the runtime's packet capture
# (deeprec_amd/_lib.py GRAPH_PACKET_CAPTURE_ENV)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_HBM_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--tables", type=int, default=26)
    p.add_argument("--rows", type=int, default=12_500_000, help="rows per table per GPU")
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--batch", type=int, default=65536, help="per-GPU batch (B_local)")
    p.add_argument("--zipf", type=float, default=0.0, help="0 = uniform keys")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=18.0)
    p.add_argument("--cpu-rows", type=int, default=12_500_000)
    p.add_argument("--check-rows", type=int, default=8192,
                   help="sampled output rows checked bit-exactly after the timed region")
    p.add_argument("--train-steps", type=int, default=10,
                   help="N=1: time the embedding training step too (0 = skip)")
    p.add_argument("--kernel-iters", type=int, default=20)
    p.add_argument("--model-steps", type=int, default=10,
                   help="timed DLRM model training steps on the headline tables (0: skip)")
    p.add_argument("--no-model-graph", dest="model_graph", action="store_false",
                   help="run the N = 1 DLRM model steps eagerly (default: one hipGraph of 4)")
    p.add_argument("--din-steps", type=int, default=10,
                   help="timed DIN (configs[3]) data-parallel training steps (0: skip)")
    p.add_argument("--din-batch", type=int, default=4096)
    p.add_argument("--no-deepfm", dest="deepfm", action="store_false",
                   help="skip the BASELINE configs[1] (DeepFM 26 x 1e7 x 64) leg at N=1")
    p.add_argument("--no-criteo", dest="criteo", action="store_false",
                   help="skip the real Criteo-TB cardinality legs (one fused table, prefix "
                        "offsets; B_local 65536 / 8192, uniform / Zipf 1.05) at N=1")
    p.add_argument("--no-dcn", dest="dcn", action="store_false",
                   help="skip the BASELINE configs[4] bf16-table leg at N=1")
    p.add_argument("--hybrid-cap", type=int, default=0,
                   help="cap the hybrid leg's large vocabularies at this many rows (rehearsals "
                        "only; 0 = the real cardinalities)")
    p.add_argument("--no-hybrid", dest="hybrid", action="store_false",
                   help="skip the real Criteo-TB cardinality leg with hybrid placement (small "
                        "features replicated, large ones row-sharded), run at every N")
    p.add_argument("--native-steps", type=int, default=32,
                   help="timed forward steps of the native C-ABI engine over RCCL (0: skip)")
    p.add_argument("--dedup", action="store_true",
                   help="xgmi engine: per-destination dedup before the exchange (grouped Unique, "
                        "unique keys routed, rows expanded locally)")
    p.add_argument("--engine", default="auto", choices=["auto", "local", "xgmi", "a2a"],
                   help="auto: local lookup at N=1, xgmi peer-write (RCCL all-to-all "
                        "fallback) at N>1; xgmi/a2a at N=1 run the sharded engine on itself")
    return p.parse_args()


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def make_batches(nb, tables, batch, keyspace, zipf, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = []
    for _ in range(nb):
        if zipf > 0:
            rng = np.random.default_rng(seed)
            k = (rng.zipf(zipf, size=(tables, batch)) - 1) % keyspace
            ids = torch.as_tensor(k, dtype=torch.int64, device=device)
        else:
            ids = torch.randint(0, keyspace, (tables, batch), generator=g, device=device,
                                dtype=torch.int64)
        out.append(ids)
        seed += 1
    return out


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args):
    """DeepRec-CPU-semantics restatement (oracle/) timed on the host cores:
    Unique -> KvResourceGather (EV hash lookup + row memcpy, Shard over
    threads) -> SparseSegmentSum, per feature, h = 1, on one table of the
    GPU's per-table shape (rows x dim), on a persistent worker pool (TF's
    CPU worker threads).  Unique is UniqueAliOp's default: ParallelComputeV1
    for N >= 14336 (unique_ali_op_util.h:651-657; serial_ = false,
    unique_ali_op.cc:55-56); the serial-Unique variant is timed beside it.
    Nine timed repeats each, interleaved; value = the best repeat (load on
    the shared host only slows a repeat down), with the median and (max -
    min) / median as the spread beside it; the id batches are drawn before
    timing.
    Threads: the box's CPU share (OMP_NUM_THREADS, else the affinity mask)."""
    from oracle import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    D, R = args.dim, args.cpu_rows
    rng = np.random.default_rng(2021)
    ev = orc.EV(D, 0.0)
    chunk = 1 << 20
    for b in range(0, R, chunk):
        keys = np.arange(b, min(R, b + chunk), dtype=np.int64)
        ev.insert(keys, rng.standard_normal((keys.shape[0], D), dtype=np.float32))
    B = args.batch
    seg_off = np.arange(B + 1, dtype=np.int32)
    out = np.empty((B, D), np.float32)
    L = orc.lib()
    pool = orc.Pool(threads)
    reps = 9   # short interleaved repeats: a few land between bursts of host load
    per = args.cpu_seconds / (2 * reps)

    batches = [rng.integers(0, R, B).astype(np.int64) for _ in range(16)]

    def timed(serial):
        done, t0, it = 0, time.perf_counter(), 0
        while True:
            ids = batches[it % len(batches)]
            it += 1
            rc = L.orc_pipeline_ev_lookup_sparse_pool(pool._h, ev._h, orc._p(ids), B,
                                                      orc._p(seg_off), B, 0, int(serial),
                                                      orc._p(out))
            assert rc == 0
            done += B
            el = time.perf_counter() - t0
            if el >= per:
                return done / el, done
    per0 = per
    per = min(0.5, per0)
    timed(False)   # warm-up: first touch of the pool's and the maps' pages
    timed(True)
    per = per0
    runs = {False: [], True: []}
    total = 0
    for _ in range(reps):   # interleaved, so drift hits both variants alike
        for serial in (False, True):
            v, n = timed(serial)
            runs[serial].append(v)
            total += n
    pool.close()
    med = {k: float(np.median(v)) for k, v in runs.items()}
    # value = the best repeat (the least disturbed: the host cores are shared
    # with other jobs, which only ever slow a repeat down -- the capacity
    # estimate that agrees across runs); the median and spread beside it
    return {"value": max(runs[False]), "median": med[False], "unit": "lookups/s",
            "cores": pool.threads, "kind": "port",
            "repeats": [round(v, 1) for v in runs[False]],
            "spread": round((max(runs[False]) - min(runs[False])) / med[False], 4),
            "serial_unique_value": max(runs[True]), "serial_unique_median": med[True],
            "serial_unique_repeats": [round(v, 1) for v in runs[True]],
            "nproc": os.cpu_count(), "cpu_model": _cpu_model(),
            "sample": "%d lookups (features of B=%d ids, h=1) over a %d-key x %d-dim fp32 EV "
                      "(one table of the GPU's per-table shape), %d x %.1f s per variant on a "
                      "persistent %d-thread pool, oracle/deeprec_oracle.c "
                      "orc_pipeline_ev_lookup_sparse_pool (UniqueAliOp's default parallel "
                      "Unique + Shard-split KvResourceGather + ali SparseSegmentSum; value = "
                      "best = the least disturbed repeat (the host is shared: load only slows "
                      "a repeat), median and spread = (max - min) / median beside it)"
                      % (total, B, R, D, reps, per, pool.threads)}


def synth_rows(seed, keys, D):
    """The bench tables' rows: synth(seed, key, col) of dr_common.h
    (SplitMix64 -> uniform [-1, 1)), for checking gathered rows."""
    M = np.uint64
    with np.errstate(over="ignore"):
        z = (M(seed) * M(0x9E3779B97F4A7C15) + keys.astype(np.uint64)[:, None] * M(0xBF58476D1CE4E5B9)
             + np.arange(D, dtype=np.uint64)[None, :] * M(0x94D049BB133111EB))
        z ^= z >> M(30)
        z *= M(0xBF58476D1CE4E5B9)
        z ^= z >> M(27)
        z *= M(0x94D049BB133111EB)
        z ^= z >> M(31)
    hi = (z >> M(32)).astype(np.uint32).view(np.int32)
    return hi.astype(np.float32) * np.float32(1.0 / 2147483648.0)


def check_rows(out, ids, T, D, n_sample, seed):
    """Sampled (bag, table) rows of a [B, T*D] sum-pooled one-hot output must
    equal the table rows synth(1000 + t, key, :) bit for bit (keys < the
    populated range); returns the number of rows checked, raises otherwise."""
    B = out.shape[0]
    rng = np.random.default_rng(seed)
    b = rng.integers(0, B, n_sample)
    t = rng.integers(0, T, n_sample)
    got = out.view(B, T, D)[torch.as_tensor(b, device=out.device),
                            torch.as_tensor(t, device=out.device)].cpu().numpy()
    keys = ids[torch.as_tensor(t, device=ids.device), torch.as_tensor(b, device=ids.device)]
    keys = keys.cpu().numpy()
    for tt in np.unique(t):
        sel = t == tt
        want = synth_rows(1000 + int(tt), keys[sel], D)
        if not np.array_equal(got[sel], want):
            bad = np.argwhere(~(got[sel] == want).all(1))[:, 0]
            raise AssertionError("headline parity: table %d, %d of %d sampled rows differ "
                                 "(first key %d)" % (tt, bad.shape[0], sel.sum(),
                                                     keys[sel][bad[0]]))
    return int(n_sample)


def _onehot_kernel_ms(feat_sets, iters, out_dtype=None):
    """Average duration of the fused one-hot EV lookup kernel over launches
    on the given feature sets in rotation (HIP events around the kernel on
    its stream, dr_kernel_timing(1))."""
    import ctypes as _C
    from deeprec_amd import _lib
    from deeprec_amd.embedding_ops import _fused_onehot
    L = _lib.lib()
    with torch.no_grad():
        for fs in feat_sets:
            assert _fused_onehot(fs, _lib.ORDER_ALI, out_dtype=out_dtype) is not None
        torch.cuda.synchronize()
        L.dr_kernel_timing(1)
        for i in range(iters):
            _fused_onehot(feat_sets[i % len(feat_sets)], _lib.ORDER_ALI, out_dtype=out_dtype)
        torch.cuda.synchronize()
        tot, cnt = _C.c_double(0.0), _C.c_int64(0)
        _lib.check(L.dr_kernel_timing_result(_C.byref(tot), _C.byref(cnt)))
        L.dr_kernel_timing(0)
    if cnt.value != iters:
        raise RuntimeError("kernel timing bracketed %d of %d launches" % (cnt.value, iters))
    return tot.value / cnt.value


def _pmc_traffic(roof, suffix, kname):
    """roofline["traffic"] (HBM bytes per launch) from the newest committed
    rocprofv3 PMC summary profiles/rNN_<suffix> of the same kernel
    (tools/pmc_summary.py: FETCH_SIZE x 2 + WRITE_SIZE, separate passes)."""
    import glob as _glob
    fs = sorted(_glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_" + suffix)))
    if not fs:
        return roof
    try:
        j = json.load(open(fs[-1]))
    except (OSError, ValueError):
        return roof
    if str(j.get("kernel", "")).startswith(kname):
        roof["traffic"] = j.get("bytes_per_launch")
        roof["traffic_source"] = os.path.relpath(fs[-1], ROOT)
        roof["traffic_round"] = os.path.basename(fs[-1])[:3]
        if roof.get("bytes_per_launch"):
            roof["traffic_ratio"] = round(j["bytes_per_launch"] / roof["bytes_per_launch"], 4)
    return roof


def _free_hbm():
    import gc
    from deeprec_amd.kv_variable_ops import flush_releases
    gc.collect()
    torch.cuda.synchronize()
    flush_releases()           # EV handles queued by __del__ (hipFree now)
    torch.cuda.empty_cache()


# Criteo-Terabyte cardinalities of the reference's SOK DLRM
# (modelzoo/SOK/DLRM/train_stand.py:242-248), looked up in ONE fused table
# with per-feature prefix offsets (model/models.py:69-76).
CRITEO_TB_VOCAB = [39884406, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 38532951, 2953546,
                   403346, 10, 2208, 11938, 155, 4, 976, 14, 39979771, 25641295, 39664984, 585935,
                   12972, 108, 36]


def criteo_legs(args, dev, log):
    """BASELINE configs[2] with the real Criteo-TB cardinalities (SURVEY 8d
    #3): the 26 features share one 1.88e8-row x 128 fp32 EV (keys = prefix
    offset + per-feature id), the fused one-hot lookup at B_local = 65 536
    and 8 192 (SOK's 65 536 / 8), uniform ids per feature and Zipf(1.05).
    lookups/s from the kernel's own launches over 4 rotating batches; the
    algorithmic bytes stay 1048 per lookup (small features hit the same rows
    again, so the HBM traffic is lower than that)."""
    import deeprec_amd as dr
    from deeprec_amd.embedding_ops import _Feature
    T, D = 26, 128
    card = np.array(CRITEO_TB_VOCAB, np.int64)
    pre = np.concatenate([[0], np.cumsum(card)[:-1]])
    total = int(card.sum())
    t0 = time.perf_counter()
    ev = dr.EmbeddingVariable("criteo_fused", D, 0.0, device=dev, capacity=total + (1 << 22))
    ev.insert_synthetic(0, total, seed=4242)
    torch.cuda.synchronize()
    log("criteo fused table: %d rows x %d in %.1fs" % (total, D, time.perf_counter() - t0))
    cardt = torch.as_tensor(card, device=dev)[None, :]
    pret = torch.as_tensor(pre, device=dev)[None, :]
    per = 8 + 16 + 2 * D * 4
    res = {"table": "one EV of %d rows x %d fp32 (26 Criteo-TB features, prefix offsets; "
                    "modelzoo/SOK/DLRM/train_stand.py:242-248, model/models.py:69-76)"
                    % (total, D), "bytes_per_lookup": per}
    for B in (65536, 8192):
        seg = torch.arange(B, dtype=torch.int32, device=dev)
        for dist_name in ("uniform", "zipf1.05"):
            recs = []
            for k in range(4):
                if dist_name == "uniform":
                    g = torch.Generator(device=dev)
                    g.manual_seed(300 + k)
                    u = torch.rand((B, T), generator=g, device=dev, dtype=torch.float64)
                    ids = (u * cardt).to(torch.int64)
                else:
                    z = np.random.default_rng(400 + k).zipf(1.05, size=(B, T)) - 1
                    ids = torch.as_tensor(z, device=dev) % cardt
                recs.append((ids + pret).contiguous())          # record-major [B, T]
            fsets = [[_Feature(ev, r[:, t], seg, B, None, "sum", None, onehot=True)
                      for t in range(T)] for r in recs]
            k_ms = _onehot_kernel_ms(fsets, args.kernel_iters)
            ach = T * B * per / (k_ms * 1e-3) / 1e9
            res["B%d_%s" % (B, dist_name)] = {
                "lookups_per_s": round(T * B / (k_ms * 1e-3), 1),
                "samples_per_s": round(B / (k_ms * 1e-3), 1), "kernel_ms": round(k_ms, 4),
                "achieved_algorithmic_GBs": round(ach, 1),
                # NOT an HBM roofline fraction: the small features' rows are
                # re-read from L2 / MALL, so the HBM bytes are below the
                # algorithmic 1 048 per lookup (no PMC traffic behind it)
                "frac_cache_inclusive": round(ach / PEAK_HBM_GBS, 4),
                "distinct_keys_batch0": int(torch.unique(recs[0]).numel())}
            log("criteo B=%d %s: %s" % (B, dist_name, json.dumps(res["B%d_%s" % (B, dist_name)])))
    dr.status_check(dev)
    del ev, fsets
    return res


class _LocalOneHot(object):
    """world 1 stand-in for a sharded engine: the fused one-hot lookup of
    its EVs (every key is local)."""

    def __init__(self, evs, batch, dev):
        from deeprec_amd.embedding_ops import SparseTensor
        self.evs = evs
        ind = torch.stack([torch.arange(batch, device=dev),
                           torch.zeros(batch, dtype=torch.int64, device=dev)], 1)
        self._sp = lambda ids: [SparseTensor(ind, ids[t], (batch, 1)) for t in range(len(evs))]

    def forward(self, ids):
        import deeprec_amd as dr
        with torch.no_grad():
            return dr.embedding_lookup_sparse_multi(self.evs, self._sp(ids), combiner="sum")

    def close(self):
        pass


def criteo_hybrid_leg(args, dev, log, world, rank, dist, staged):
    """The real Criteo-TB cardinalities at N GPUs with hybrid placement
    (sharded.HybridShardedLookup): the 20 features of <= 585 935 rows
    (1.11 M rows, 0.57 GB) are replicated on every rank and looked up
    locally -- one fused one-hot kernel over their prefix-offset table, on a
    side stream -- and the 6 large ones (1.87e8 rows) are row-sharded (key %
    N) and exchanged by the xGMI peer-write engine (RCCL all-to-all
    fallback).  B_local ids per feature per rank, uniform over the feature's
    vocabulary.  value = 26 * B_local * N / step time (barrier-bracketed,
    max over ranks).  At N = 1 both parts are local lookups (the same code
    path, no exchange)."""
    import deeprec_amd as dr
    from deeprec_amd import _lib
    from deeprec_amd.embedding_ops import _Feature, _fused_onehot
    from deeprec_amd.sharded import (HybridShardedLookup, ShardedLookup, XgmiShardedLookup,
                                     hybrid_split)
    D, B = 128, args.batch
    card = np.array(CRITEO_TB_VOCAB, np.int64)
    rep, shard = hybrid_split(CRITEO_TB_VOCAB, 585935)
    if args.hybrid_cap > 0:
        card[shard] = np.minimum(card[shard], args.hybrid_cap)
    rcard = card[rep]
    rpre = np.concatenate([[0], np.cumsum(rcard)[:-1]])
    t0 = time.perf_counter()
    rep_ev = dr.EmbeddingVariable("hyb_rep", D, 0.0, device=dev,
                                  capacity=int(rcard.sum()) + (1 << 20))
    rep_ev.insert_synthetic(0, int(rcard.sum()), seed=4242)
    sh_evs = []
    for t in shard:
        n_own = int((card[t] - rank + world - 1) // world)
        ev = dr.EmbeddingVariable("hyb_sh%d" % t, D, 0.0, device=dev,
                                  capacity=n_own + max(1 << 20, 4 * world * B))
        ev.insert_synthetic(rank, n_own, seed=5000 + t, key_stride=world)
        sh_evs.append(ev)
    torch.cuda.synchronize()
    log("hybrid tables: replicated %d features / %d rows, sharded %d features / %d rows "
        "per rank, in %.1fs" % (len(rep), int(rcard.sum()), len(shard),
                                sum(int(e.total_count()[0]) for e in sh_evs),
                                time.perf_counter() - t0))
    kind = "local (N=1)"
    a2a = None
    if world == 1:
        engine = _LocalOneHot(sh_evs, B, dev)
    else:
        engine, ok, err = None, 1, ""
        try:
            barrier = None
            if staged:
                def barrier():
                    torch.cuda.synchronize()
                    dist.barrier()
            engine = XgmiShardedLookup(sh_evs, world, rank, B, dev, barrier=barrier)
        except Exception as e:  # noqa: BLE001
            ok, err = 0, str(e)
        flag = torch.tensor([ok], dtype=torch.int32, device="cpu" if staged else dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        a2a = ShardedLookup(sh_evs, world, rank, B, dev)
        if staged:
            def staged_a2a(out, inp, out_splits=None, in_splits=None):
                o = torch.empty(out.shape, dtype=out.dtype)
                dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
                out.copy_(o)
                return out
            a2a._a2a = staged_a2a
        if int(flag.item()) == 1:
            kind = "xgmi peer-write"
        else:
            log("hybrid: xgmi unavailable (%s); RCCL all-to-all" % err)
            if engine is not None:
                engine.close()
            engine, kind = a2a, "RCCL all-to-all"
    seg = torch.arange(B, dtype=torch.int32, device=dev)
    cardt = torch.as_tensor(card, device=dev)[:, None]
    fsets, ishard, idsall = [], [], []
    for k in range(4):
        g = torch.Generator(device=dev)
        g.manual_seed(600 + 7919 * rank + k)
        u = torch.rand((26, B), generator=g, device=dev, dtype=torch.float64)
        ids = (u * cardt).to(torch.int64)                     # [26, B] per-feature ids
        idsall.append(ids)
        rrec = (ids[rep] + torch.as_tensor(rpre, device=dev)[:, None]).t().contiguous()
        fsets.append([_Feature(rep_ev, rrec[:, j], seg, B, None, "sum", None, onehot=True)
                      for j in range(len(rep))])
        ishard.append(ids[shard].contiguous())

    def local_lookup(fs):
        return _fused_onehot(fs, _lib.ORDER_ALI)

    hyb = HybridShardedLookup(local_lookup, engine, dev, overlap=True)

    def step(k):
        return hyb.forward(fsets[k % 4], ishard[k % 4])

    with torch.no_grad():
        for w in range(max(args.warmup, 2)):
            out_r, out_s = step(w)
            torch.cuda.synchronize()
        # correctness (outside the timing): sampled rows of both blocks are
        # the tables' synth rows; at N > 1 the exchange equals the all-to-all
        # engine's output bit for bit
        checked, ok_rows = 0, True
        for k in range(2):
            out_r, out_s = step(k)
            out_r, out_s = out_r.clone(), out_s.clone()
            ids = idsall[k].cpu().numpy()
            rs = np.random.default_rng(31 + k).integers(0, B, 64)
            for j, t in enumerate(rep):
                want = synth_rows(4242, ids[t, rs] + rpre[j], D)
                ok_rows &= np.array_equal(out_r[rs, j * D:(j + 1) * D].cpu().numpy(), want)
                checked += rs.size
            for j, t in enumerate(shard):
                want = synth_rows(5000 + t, ids[t, rs], D)
                ok_rows &= np.array_equal(out_s[rs, j * D:(j + 1) * D].cpu().numpy(), want)
                checked += rs.size
            if a2a is not None and engine is not a2a:
                ok_rows &= bool(torch.equal(out_s, a2a.forward(ishard[k])))
        if world > 1:
            f = torch.tensor([int(ok_rows)], dtype=torch.int32, device="cpu" if staged else dev)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            ok_rows = bool(f.item())
        dr.status_check(dev)
        if not ok_rows:
            raise AssertionError("hybrid leg: rows differ from the tables' synth rows / a2a")
        for i in range(args.warmup):
            step(i)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # each part alone (same batches, same barriers): the replicated
        # features' local lookup, then the sharded features' lookup with its
        # exchange -- the inputs of DESIGN section 7's model
        parts = []
        for fn in (lambda i: local_lookup(fsets[i % 4]), lambda i: engine.forward(ishard[i % 4])):
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            tp = time.perf_counter()
            for i in range(args.steps):
                fn(i)
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            parts.append(time.perf_counter() - tp)
    if dist is not None:
        te = torch.tensor([el] + parts, dtype=torch.float64, device="cpu" if staged else dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        el, parts = float(te[0].item()), [float(x) for x in te[1:].tolist()]
    ms = el / args.steps * 1e3
    res = {"workload": "real Criteo-TB cardinalities (modelzoo/SOK/DLRM/train_stand.py:242-248), "
                       "hybrid placement: %d features <= 585935 rows replicated (one fused "
                       "%d-row table, local fused lookup on a side stream), %d large features "
                       "row-sharded key %% N (%s exchange), B_local=%d, uniform ids per feature, "
                       "embedding_lookup_sparse(sum) forward" % (len(rep), int(rcard.sum()),
                                                                 len(shard), kind, B),
           "n_gpus": world, "ms_per_step": round(ms, 4),
           "parts_ms_per_step": {"replicated_local": round(parts[0] / args.steps * 1e3, 4),
                                 "sharded_with_exchange": round(parts[1] / args.steps * 1e3, 4)},
           "lookups_per_s": round(26 * B * world / (ms * 1e-3), 1),
           "samples_per_s": round(B * world / (ms * 1e-3), 1),
           "sharded_lookups_per_gpu_step": len(shard) * B,
           "remote_rows_per_gpu_step": int(len(shard) * B * (world - 1) / world),
           "engine": kind, "checked_rows": checked, "bitexact": True,
           "vocab_cap": args.hybrid_cap or None}
    log("criteo hybrid leg: %s" % json.dumps(res))
    if hasattr(engine, "close"):
        engine.close()
    return res


def _state(model, evs):
    """Parameters and EV contents (sorted by key) of a model, for bit compares."""
    ps = [p.detach().clone() for p in model.parameters()]
    es = []
    for ev in evs:
        k, v = ev.export()[:2]
        o = torch.argsort(k)
        es.append((k[o], v[o]))
    return ps, es


def _same_state(a, b):
    (pa, ea), (pb, eb) = a, b
    return (all(torch.equal(x.view(torch.int32), y.view(torch.int32)) for x, y in zip(pa, pb))
            and all(torch.equal(ka, kb) and torch.equal(va.view(torch.int32), vb.view(torch.int32))
                    for (ka, va), (kb, vb) in zip(ea, eb)))


def _ev_rows_io(evs, rowsets, D, saved=None):
    """Copy the given rows (int32 row indices) of fp32 EVs out of their pools
    (saved=None: returns the copies) or back in (dr_rows_pack / _scatter on
    the pool pointer)."""
    import ctypes as _C
    from deeprec_amd._lib import check, lib, ptr, stream_handle
    out = []
    for i, (ev, r) in enumerate(zip(evs, rowsets)):
        pool, st = _C.c_void_p(ev.pool()), stream_handle(r.device)
        if saved is None:
            o = torch.empty((r.numel(), D), dtype=torch.float32, device=r.device)
            check(lib().dr_rows_pack(pool, ptr(r), r.numel(), None, D, ptr(o), st))
            out.append(o)
        else:
            check(lib().dr_rows_scatter(ptr(saved[i]), ptr(r), r.numel(), None, D, pool, st))
    return out


def _dlrm_graph_check(mgraph, glosses, mstep, model, evs, idlist, D, n, rounds=2):
    """The captured n DLRM steps (SGD dense + KV) against n eager steps from
    the same state: parameters and the EV rows of every key the batches touch
    are saved, the eager steps run, their losses / parameters / rows are kept,
    the state is put back and the graph replayed -- `rounds` times, eager work
    in between -- each replay bit-compared with the eager result."""
    keys = [torch.unique(torch.cat([ids[t] for ids in idlist])) for t in range(len(evs))]
    rows = [ev.resolve(k).to(torch.int32) for ev, k in zip(evs, keys)]
    params = list(model.parameters())
    p0 = [p.detach().clone() for p in params]
    r0 = _ev_rows_io(evs, rows, D)
    le = [mstep(i).detach().clone() for i in range(n)]
    pe = [p.detach().clone() for p in params]
    re_ = _ev_rows_io(evs, rows, D)
    eq = lambda a, b: torch.equal(a.view(torch.int32), b.view(torch.int32))  # noqa: E731
    for rep in range(rounds):
        with torch.no_grad():
            for p, v in zip(params, p0):
                p.copy_(v)
        _ev_rows_io(evs, rows, D, r0)
        mgraph.replay()
        torch.cuda.synchronize()
        bad = [i for i in range(n) if not eq(glosses[i].detach(), le[i])]
        if bad:
            return "replay %d: step %d loss %r != eager %r" % (rep, bad[0], float(glosses[bad[0]]),
                                                                float(le[bad[0]]))
        if not all(eq(p.detach(), v) for p, v in zip(params, pe)):
            return "replay %d: parameters differ from the eager steps" % rep
        if not all(eq(a, b) for a, b in zip(_ev_rows_io(evs, rows, D), re_)):
            return "replay %d: EV rows differ from the eager steps" % rep
        # eager work between the replays (what the runtime bug needed)
        junk = [torch.full((int(k),), float("nan"), device=p0[0].device)
                for k in torch.randint(1, 1 << 18, (500,)).tolist()]
        del junk
    return "equal: %d replays of %d steps from a restored state, losses + parameters + %d " \
           "touched EV rows bit-equal to the eager steps" % (rounds, n,
                                                              sum(int(r.numel()) for r in rows))


def _din_graph_check(graphs, glosses, shadow_step, cur, shadow, dev, rounds=2):
    """Replay the captured steps `rounds` times over, an eager shadow step of
    the same batch before each replay; returns "equal ..." when every loss
    and, at the end, every parameter and EV row agree bit for bit."""
    n = 0
    for _ in range(rounds):
        for j, gr in enumerate(graphs):
            le = shadow_step(j).detach()
            gr.replay()
            torch.cuda.synchronize()
            if not torch.equal(le.view(torch.int32), glosses[j].detach().view(torch.int32)):
                return "replay %d (graph %d) loss %r != eager shadow %r" % (
                    n, j, float(glosses[j]), float(le))
            n += 1
    evs_c, model_c = cur
    evs_s, model_s = shadow
    if not _same_state(_state(model_c, evs_c), _state(model_s, evs_s)):
        return "parameters / EV rows differ from the eager shadow after %d replays" % n
    return "equal: %d replays interleaved with eager shadow steps, losses + parameters + EV " \
           "rows bit-equal" % n


def din_leg(args, dev, log, world, rank, dist, staged):
    """BASELINE configs[3]: DIN (modelzoo/DIN/script/model.py) at B_local =
    4096, histories U[1, 100] padded to the batch max, dim 18, vocabularies
    5e5 users / 4e5 items / 2e3 categories, Adam (dense and KV).  At N > 1
    data parallel over replicated EVs (modelzoo.din_train_step(world=N):
    dense gradients all-reduced, EV gradient slices gathered in rank order);
    each rank its own batch.  Eager, barrier-bracketed, max over ranks."""
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    B, T, D = args.din_batch, 100, 18
    R = (500_000, 400_000, 2_000)
    # one GPU: the step as hipGraphs, one per batch shape (DR_DIN_GRAPH=0:
    # eager); capturable dense Adam (step counts on the device), KV Adam's
    # beta powers in HBM (training.AdamOptimizer._device_powers).  Before the
    # graphs are timed they are checked against an eager shadow model (same
    # seeds, same steps) stepped BETWEEN the replays in this process -- the
    # interleaving that broke round 5's replays (the runtime's graph packet
    # capture, deeprec_amd/_lib.py) -- over two rounds of the four graphs;
    # any bit that differs and the eager step is timed instead
    use_graph = (world == 1 and getattr(args, "model_graph", True)
                 and os.environ.get("DR_DIN_GRAPH", "1") == "1")

    def make(tag):
        evs = []
        for i, r in enumerate(R):
            ev = dr.EmbeddingVariable("din_%s%d" % (tag, i), D, 0.0, capacity=r + (1 << 16),
                                      device=dev)
            ev.insert_synthetic(0, r, seed=700 + i)
            evs.append(ev)
        torch.manual_seed(0)
        model = mz.DIN(*evs).to(dev)
        # the dense Adam as torch's fused kernel (one launch per step instead
        # of ~15 multi-tensor launches; DR_BENCH_DENSE_ADAM=foreach: A/B)
        fused = os.environ.get("DR_BENCH_DENSE_ADAM", "fused") == "fused"
        dopt = torch.optim.Adam(model.parameters(), lr=0.001, capturable=use_graph,
                                fused=fused or None)
        return evs, model, dopt, dr.AdamOptimizer(0.001)
    evs, model, dopt, eopt = make("b")
    shadow = make("s") if use_graph else None
    g = torch.Generator(device=dev)
    g.manual_seed(2021 + 7919 * rank)
    batches = []
    for _ in range(4):
        lens = torch.randint(1, T + 1, (B,), generator=g, device=dev)
        Tb = int(lens.max())
        mask = (torch.arange(Tb, device=dev)[None, :] < lens[:, None]).float()
        mh = torch.randint(1, R[1], (B, Tb), generator=g, device=dev) * mask.long()
        ch = torch.randint(1, R[2], (B, Tb), generator=g, device=dev) * mask.long()
        lab = (torch.rand(B, generator=g, device=dev) > 0.5).long()
        batches.append((torch.randint(0, R[0], (B,), generator=g, device=dev),
                        torch.randint(0, R[1], (B,), generator=g, device=dev),
                        torch.randint(0, R[2], (B,), generator=g, device=dev), mh, ch, mask,
                        torch.stack([lab, 1 - lab], 1).float()))

    def dstep(i, m=None, stamp=True):
        # stamp=False: no global step reaches the EV apply (a captured graph
        # would replay its capture-time step as every row's version; these
        # EVs have steps_to_live = 0, so no version is kept either way)
        e_, md, do, eo = m or (evs, model, dopt, eopt)
        return mz.din_train_step(md, batches[i % 4], do, eo, i if stamp else None, world=world,
                                 staged=staged)

    for i in range(4 if use_graph else 2):   # graphs: every batch shape once first
        dstep(i)
        if shadow is not None:
            dstep(i, shadow)
    torch.cuda.synchronize()
    dr.status_check(dev)
    graphs, graph_err, eager_ms, graph_check = None, None, None, None
    if use_graph:
        t0 = time.perf_counter()
        for i in range(4, 4 + args.din_steps):
            dstep(i)
        torch.cuda.synchronize()
        eager_ms = (time.perf_counter() - t0) / args.din_steps * 1e3
        for i in range(4, 4 + args.din_steps):
            dstep(i, shadow)
        try:
            for m in (evs, shadow[0]):   # a captured resolve must not be able to outgrow the table
                for ev in m:
                    ev.reserve(8 * B * (T + 1))   # 4 graphs x (lookup + apply) adds, counted conservatively
            torch.cuda.synchronize()
            graphs, glosses = [], []
            pool = torch.cuda.graph_pool_handle()
            for j in range(4):
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, pool=pool):
                    glosses.append(dstep(j, stamp=False))
                graphs.append(gr)
            graph_check = _din_graph_check(graphs, glosses, lambda j: dstep(j, shadow, False),
                                           (evs, model), shadow[:2], dev)
            dr.status_check(dev)
            if not graph_check.startswith("equal"):
                graph_err, graphs = graph_check, None
        except Exception as e:   # report the eager step instead
            graphs, graph_err = None, "%s: %s" % (type(e).__name__, str(e)[:200])
            torch.cuda.synchronize()
        shadow = None
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.din_steps):
        if graphs is not None:
            graphs[i % 4].replay()
        else:
            dstep(i)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist is not None:
        te = torch.tensor([el], dtype=torch.float64, device="cpu" if staged else dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        el = float(te.item())
    dr.status_check(dev)
    ms = el / args.din_steps * 1e3
    res = {"workload": "BASELINE configs[3] DIN: B_local=%d, histories U[1, %d], dim %d, vocab "
                       "%s, Adam; %s" % (B, T, D, list(R), "data parallel over replicated EVs "
                                         "(dense all-reduce + EV gradient slices gathered)"
                                         if world > 1 else "one GPU"),
           "n_gpus": world, "ms_per_step": round(ms, 4), "global_batch": world * B,
           "samples_per_s": round(world * B / (ms * 1e-3), 1), "steps": args.din_steps,
           "hipgraph": graphs is not None}
    if eager_ms is not None:
        res["ms_per_step_eager"] = round(eager_ms, 4)
    if graph_check:
        res["graph_check"] = graph_check
    if graph_err:
        res["graph_error"] = graph_err
    log("din leg: %s" % json.dumps(res))
    return res


def lookup_kernel_label(G):
    """The fused one-hot lookup the library launches for G lanes per row
    (DR_LOOKUP_KERNEL, ev.hip lookup_kernel_kind(); default 1 = line probes)."""
    kind = os.environ.get("DR_LOOKUP_KERNEL", "1")
    if kind == "0":
        return "dr::ev_lookup_onehot_kernel<4,%d,1,ALI,%d>" % (G, 2 if G <= 16 else 4)
    name = "ev_lookup_line_kernel" if kind == "1" else "ev_lookup_pipe_kernel"
    return "dr::%s<4,%d,1,ALI>" % (name, G)


def dcn_bf16_leg(args, dev, log):
    """BASELINE configs[4] per-GPU embedding shape with bf16 tables: 26 bf16
    EVs x 12.5 M rows x 128, B = 65 536, the fused one-hot lookup writing
    the bf16 [B, 26*128] CrossNet input bitwise (8 key + 16 slot + 256 row
    + 256 out bytes per lookup), and the embedding training step on those
    tables (fp32 gradients, SGD rounding each updated value to bf16)."""
    import deeprec_amd as dr
    from deeprec_amd.embedding_ops import SparseTensor, _Feature
    T, D, R, B = 26, 128, 12_500_000, args.batch
    evs = []
    t0 = time.perf_counter()
    for t in range(T):
        ev = dr.EmbeddingVariable("dcn%d" % t, D, 0.0, device=dev, capacity=R + (1 << 20),
                                  value_dtype=torch.bfloat16)
        ev.insert_synthetic(0, R, seed=6000 + t)
        evs.append(ev)
    torch.cuda.synchronize()
    log("dcn bf16 tables in %.1fs" % (time.perf_counter() - t0))
    batches = make_batches(4, T, B, R, 0.0, 91, dev)
    recs = [ids.t().contiguous() for ids in batches]
    seg = torch.arange(B, dtype=torch.int32, device=dev)
    fsets = [[_Feature(evs[t], r[:, t], seg, B, None, "sum", None, onehot=True) for t in range(T)]
             for r in recs]
    k_ms = _onehot_kernel_ms(fsets, args.kernel_iters, out_dtype=torch.bfloat16)
    per = 8 + 16 + 2 * D * 2
    ach = T * B * per / (k_ms * 1e-3) / 1e9
    # parity at this size: sampled rows of one output == bf16(synth) bitwise
    from deeprec_amd.embedding_ops import _fused_onehot
    from deeprec_amd import _lib
    with torch.no_grad():
        out = _fused_onehot(fsets[0], _lib.ORDER_ALI, out_dtype=torch.bfloat16)
    rng = np.random.default_rng(3)
    bs, ts = rng.integers(0, B, 2048), rng.integers(0, T, 2048)
    got = out.view(B, T, D)[torch.as_tensor(bs, device=dev), torch.as_tensor(ts, device=dev)]
    got = got.view(torch.int16).cpu().numpy().view(np.uint16)
    keys = recs[0][torch.as_tensor(bs, device=dev), torch.as_tensor(ts, device=dev)].cpu().numpy()
    for tt in np.unique(ts):
        sel = ts == tt
        w = synth_rows(6000 + int(tt), keys[sel], D)
        wb = ((w.view(np.uint32) + np.uint32(0x7FFF) + ((w.view(np.uint32) >> 16) & 1)) >> 16)
        if not np.array_equal(got[sel], wb.astype(np.uint16)):
            raise AssertionError("dcn bf16 leg: table %d rows differ from bf16(synth)" % tt)
    ind = torch.stack([torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64, device=dev)],
                      1)
    sps = [[SparseTensor(ind, ids[t], (B, 1)) for t in range(T)] for ids in batches]
    opt = dr.GradientDescentOptimizer(0.01)
    up = torch.randn((B, T * D), device=dev).to(torch.bfloat16)

    def tstep(i):
        o = dr.embedding_lookup_sparse_multi(evs, sps[i % 4], combiner="sum",
                                             out_dtype=torch.bfloat16)
        o.backward(up)
        opt.apply_gradients(evs)

    for i in range(2):
        tstep(i)
    torch.cuda.synchronize()
    for ev in evs:
        ev.reserve(8 * B)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(4):
            tstep(i)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = max(1, args.train_steps // 4)
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    tms = (time.perf_counter() - t0) / (4 * reps) * 1e3
    dr.status_check(dev)
    res = {"workload": "BASELINE configs[4] per-GPU embedding shape: 26 bf16 EV tables x %d rows "
                       "x %d, B=%d, hotness 1, uniform keys, fused one-hot lookup into the bf16 "
                       "CrossNet input (DR_LOOKUP_OUT_BF16)" % (R, D, B),
           "lookups_per_s": round(T * B / (k_ms * 1e-3), 1),
           "samples_per_s": round(B / (k_ms * 1e-3), 1),
           "checked_rows": 2048,
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS,
                        "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4),
                        "kernel": lookup_kernel_label(16) + " on bf16 rows (64 float words)",
                        "kernel_ms": round(k_ms, 4), "bytes_per_lookup": per,
                        "bytes_per_launch": T * B * per},
           "train_step": {"ms_per_step": round(tms, 4),
                          "samples_per_s": round(B / (tms * 1e-3), 1),
                          "step": "fused bf16 lookup recording rows + row-grouped backward (fp32 "
                                  "gradients) fused with the KV SGD update rounding to bf16 "
                                  "(dr_ev_pool_grad_rows_apply_sgd), hipGraph of 4 steps"}}
    _pmc_traffic(res["roofline"], "pmc_traffic_dcn.json", "ev_lookup_line_kernel")
    log("dcn bf16 leg: %s" % json.dumps(res))
    del evs, fsets, g
    return res


def deepfm_leg(args, dev, log):
    """BASELINE configs[1] (DeepFM: 26 tables x 1e7 rows x 64 fp32, one
    MI355X): the fused one-hot EV lookup on its own table shape -- lookups/s,
    the kernel's HBM roofline (8 key + 16 slot + 256 row + 256 out bytes per
    lookup) and the embedding-layer training step (SGD), on uniform keys.
    Runs after the headline's tables are freed (both sets do not fit 288 GB
    together)."""
    import deeprec_amd as dr
    from deeprec_amd import _lib
    from deeprec_amd.embedding_ops import SparseTensor, _Feature, _fused_onehot
    T, D, R, B = 26, 64, 10_000_000, args.batch
    evs = []
    for t in range(T):
        ev = dr.EmbeddingVariable("deepfm%d" % t, D, 0.0, device=dev, capacity=R + (1 << 20))
        ev.insert_synthetic(0, R, seed=5000 + t)
        evs.append(ev)
    batches = make_batches(4, T, B, R, 0.0, 77, dev)
    recs = [ids.t().contiguous() for ids in batches]      # record-major [B, T], as main()
    seg = torch.arange(B, dtype=torch.int32, device=dev)
    # the kernel's own launches over the four batches in rotation (as main())
    import ctypes as _C
    L = _lib.lib()
    with torch.no_grad():
        kfeats = [[_Feature(evs[t], r[:, t], seg, B, None, "sum", None, onehot=True)
                   for t in range(T)] for r in recs]
        for fs in kfeats:
            _fused_onehot(fs, _lib.ORDER_ALI)
        torch.cuda.synchronize()
        L.dr_kernel_timing(1)
        for i in range(args.kernel_iters):
            _fused_onehot(kfeats[i % len(kfeats)], _lib.ORDER_ALI)
        torch.cuda.synchronize()
        tot, cnt = _C.c_double(0.0), _C.c_int64(0)
        _lib.check(L.dr_kernel_timing_result(_C.byref(tot), _C.byref(cnt)))
        L.dr_kernel_timing(0)
    k_ms = tot.value / max(cnt.value, 1)
    per = 8 + 16 + 2 * D * 4
    ach = T * B * per / (k_ms * 1e-3) / 1e9
    # embedding-layer training step, hipGraph of 4 steps as in main()
    ind = torch.stack([torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64, device=dev)],
                      1)
    sps = [[SparseTensor(ind, ids[t], (B, 1)) for t in range(T)] for ids in batches]
    opt = dr.GradientDescentOptimizer(0.01)
    up = torch.randn((B, T * D), device=dev)

    def tstep(i):
        out = dr.embedding_lookup_sparse_multi(evs, sps[i % 4], combiner="sum")
        out.backward(up)
        opt.apply_gradients(evs)

    for i in range(2):
        tstep(i)
    torch.cuda.synchronize()
    for ev in evs:
        ev.reserve(8 * B)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(4):
            tstep(i)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = max(1, args.train_steps // 4)
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    tms = (time.perf_counter() - t0) / (4 * reps) * 1e3
    dr.status_check(dev)
    res = {"workload": "BASELINE configs[1] DeepFM shape: 26 EV tables x %d rows x %d fp32, "
                       "B=%d, hotness 1, uniform keys, fused one-hot embedding_lookup_sparse(sum)"
                       % (R, D, B),
           "lookups_per_s": round(T * B / (k_ms * 1e-3), 1),
           "samples_per_s": round(B / (k_ms * 1e-3), 1),
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS,
                        "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4),
                        "kernel": lookup_kernel_label(16),
                        "kernel_ms": round(k_ms, 4), "bytes_per_lookup": per,
                        "bytes_per_launch": T * B * per},
           "train_step": {"ms_per_step": round(tms, 4),
                          "samples_per_s": round(B / (tms * 1e-3), 1),
                          "step": "fused lookup recording rows + row-grouped backward fused with "
                                  "the KV SGD update (dr_ev_pool_grad_rows_apply_sgd), hipGraph "
                                  "of 4 steps"}}
    _pmc_traffic(res["roofline"], "pmc_traffic_deepfm.json", "ev_lookup_line_kernel")
    log("deepfm leg: %s" % json.dumps(res))
    del evs, kfeats, g
    return res


def exchange_phases(ph, batches, world, rank, T, D, dist, staged, dev):
    """Per-step phase times of the peer-write engine (this rank and the max
    over ranks) with its link traffic: rows this rank serves to remote
    requesters (owner side, exact from every rank's id counts per owner),
    rows it receives, and the achieved xGMI write rate of its serve phase."""
    if ph is None:
        return None
    cnt = torch.zeros(world, dtype=torch.float64, device=dev)
    for ids in batches:
        cnt += torch.bincount((ids % world).reshape(-1), minlength=world).double()
    cnt /= len(batches)                    # ids this rank sends to each owner per step
    sent = cnt.clone()
    sent[rank] = 0.0
    tot = sent.cpu() if staged else sent.clone()
    dist.all_reduce(tot)                   # tot[d]: remote ids owner d serves per step
    row_bytes = D * 4
    out_rows = float(tot[rank])
    in_rows = float(sent.sum())
    names = ("route", "wait_route", "serve", "wait_serve")
    mx = torch.tensor([ph[k] for k in names], dtype=torch.float64,
                      device="cpu" if staged else dev)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    res = {"ms_rank0" if rank == 0 else "ms_this_rank": {k: round(ph[k], 4) for k in names},
           "ms_max_over_ranks": {k: round(float(mx[i]), 4) for i, k in enumerate(names)},
           "steps": ph["steps"],
           "remote_rows_served_per_step": int(round(out_rows)),
           "remote_rows_received_per_step": int(round(in_rows)),
           "link_bytes_out_per_step": int(round(out_rows * row_bytes)),
           "xgmi_write_GBps_serve_phase": round(out_rows * row_bytes / (ph["serve"] * 1e-3) / 1e9, 1),
           "xgmi_write_GBps_per_link": round(out_rows * row_bytes / max(world - 1, 1) /
                                             (ph["serve"] * 1e-3) / 1e9, 1),
           "note": "serve = owner insert-on-miss resolve + every row written to its requester "
                   "over xGMI (the link-bound phase); wait_* = stream-ordered barrier (slowest "
                   "peer + collective latency)"}
    return res


def native_rccl_leg(args, evs, batches, engine, a2a, local_step, world, rank, dist, staged, dev,
                    log):
    """NativeShardedLookup over Comm.rccl (the library's sharded C entries on
    the RCCL transport; Comm.host_staged in a gloo rehearsal), each engine
    kind of dr_sharded_create_ex: "rccl" (exact-size all-to-alls, the split
    sizes read on the host), "xgmi" (peer writes into IPC-mapped buffers,
    barriers through the comm, the result left in the engine's buffer -- no
    host read) and, at N = 1, "fixed" (all-to-alls at fixed capacity, no
    host read; it moves N x the keys at N > 1).  Each kind's output checked
    bit for bit against the all-to-all engine (N > 1) or the local fused
    lookup (N = 1), then timed forward-only."""
    from deeprec_amd.sharded import Comm, NativeShardedLookup
    T, B = args.tables, args.batch
    comm = Comm.host_staged() if staged else Comm.rccl(rank, world)
    kinds = ["xgmi", "rccl"] + (["fixed"] if world == 1 else [])
    out = {"transport": "gloo host-staged callback (rehearsal)" if staged else
           "RCCL (dr_comm_init with an ncclUniqueId)"}
    n = args.native_steps
    for kind in kinds:
        try:
            eng = NativeShardedLookup(comm, evs, dev, kind=kind, batch=B, max_ids=B)
        except Exception as e:  # noqa: BLE001 -- one kind must not cost the others
            out[kind] = {"error": str(e)[:200]}
            continue
        copy = kind != "xgmi"   # xgmi: the result stays in the engine buffer
        same = 1
        with torch.no_grad():
            for k in range(len(batches)):
                got = eng.forward(batches[k], combiner="sum", copy=copy).clone()
                ref = a2a.forward(batches[k]) if a2a is not None else local_step(k)
                same &= int(torch.equal(got, ref))
        if world > 1:
            flag = torch.tensor([same], dtype=torch.int32, device="cpu" if staged else dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            same = int(flag.item())
        # one GPU, host-read-free kinds: the forward as a hipGraph (as the
        # headline step), kept only if every batch's replay equals the local
        # lookup bit for bit (DR_NATIVE_GRAPH=0: eager)
        graph, static, graph_note = None, None, None
        if (world == 1 and not staged and kind in ("xgmi", "fixed")
                and os.environ.get("DR_NATIVE_GRAPH", "1") == "1"):
            try:
                with torch.no_grad():
                    for e_ in evs:   # a captured serve must not be able to grow a table
                        e_.reserve(2 * B * world)
                    torch.cuda.synchronize()
                    static = batches[0].clone()
                    s = torch.cuda.Stream()
                    s.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s):
                        eng.forward(static, combiner="sum", copy=copy)
                    torch.cuda.current_stream().wait_stream(s)
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr):
                        gout = eng.forward(static, combiner="sum", copy=copy)
                    ok = True
                    for k in range(len(batches)):
                        static.copy_(batches[k])
                        gr.replay()
                        torch.cuda.synchronize()
                        ok = ok and torch.equal(gout, local_step(k))
                    graph = gr if ok else None
                    graph_note = None if ok else "replay != local lookup: eager timed"
            except Exception as e:  # noqa: BLE001 -- time the eager forward instead
                graph, graph_note = None, "capture failed (%s: %s): eager timed" % (
                    type(e).__name__, str(e)[:160])
                torch.cuda.synchronize()
        with torch.no_grad():
            for k in range(2):
                if graph is not None:
                    static.copy_(batches[k])
                    graph.replay()
                else:
                    eng.forward(batches[k], combiner="sum", copy=copy)
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                if graph is not None:
                    static.copy_(batches[i % len(batches)])
                    graph.replay()
                else:
                    eng.forward(batches[i % len(batches)], combiner="sum", copy=copy)
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el], dtype=torch.float64, device="cpu" if staged else dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        st = eng.stats()
        graphed = graph is not None
        graph = static = None   # the graph holds the engine's buffers: drop it first
        torch.cuda.synchronize()
        eng.close()
        res = {"engine_check": "native C-ABI engine (%s) == %s, %d batches, all ranks: %s" % (
                   kind, "all-to-all engine" if a2a is not None else "local fused lookup",
                   len(batches), bool(same)),
               "ms_per_step": round(el / n * 1e3, 4), "steps": n, "graph": graphed,
               "graph_note": graph_note,
               "lookups_per_s": round(T * B * world * n / el, 1),
               "note": {"rccl": "reads the per-peer split sizes on the host once per step",
                        "xgmi": "route -> barrier -> owner serve (peer writes) -> barrier, "
                                "no host read; output left in the engine buffer",
                        "fixed": "fixed-capacity all-to-alls, device counts, no host read"}[kind]}
        if kind == "rccl":
            res["sent_keys_last_step"] = st["sent_keys"]
            res["recv_keys_last_step"] = st["recv_keys"]
        out[kind] = res
        log("native engine %s: %s" % (kind, json.dumps(res)))
    comm.close()
    return out


def main():
    args = parse()
    import deeprec_amd as dr
    from deeprec_amd import _lib, ops
    from deeprec_amd.embedding_ops import SparseTensor

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DR_BENCH_GLOO_STAGED=1: rehearsal of the N>1 path with every rank on
    # cuda:0 and the all-to-alls staged through host memory over gloo (a
    # 1-GPU box cannot host two RCCL ranks).  Never used for reported numbers.
    staged = world > 1 and os.environ.get("DR_BENCH_GLOO_STAGED") == "1"
    if staged:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if staged:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    dr.load()
    T, D, B, R = args.tables, args.dim, args.batch, args.rows
    torch.cuda.synchronize()

    # ---- tables: T EVs, keys [0, R) resident with synthetic rows ---------
    t0 = time.perf_counter()
    evs = []
    for t in range(T):
        # headroom for the worst-case new keys of the steps in flight before
        # the asynchronously mirrored row count catches up: B (local
        # resolve) or N * B (an owner serving every rank, dr_xgmi_serve) per
        # step, 4 steps' worth (a lagging mirror past that costs one host
        # sync, never a growth: every key here exists).  Row pool = capacity
        # rows, key table next_pow2(2 x capacity) slots: at N = 8 and
        # B = 65 536 that is 14.6 M rows (7.5 GB) + 33.5 M slots (0.54 GB)
        # per table, against 18.8 M / 67 M with the earlier 12 x N x B.
        ev = dr.EmbeddingVariable("table%d" % t, D, 0.0, device=dev,
                                  capacity=R + max(1 << 20, 4 * world * B))
        # rank r owns keys k % world == r of the keyspace [0, R * world)
        ev.insert_synthetic(rank, R, seed=1000 + t, key_stride=world)
        evs.append(ev)
    torch.cuda.synchronize()
    log("populated %d EVs x %d rows x %d dim in %.1fs" % (T, R, D, time.perf_counter() - t0))

    engine_kind = "local"
    want = args.engine if args.engine != "auto" else ("local" if world == 1 else "xgmi")
    if want != "local":
        from deeprec_amd.sharded import ShardedLookup, XgmiShardedLookup
        keyspace = R * world
        engine = None
        if want == "xgmi" and world == 1:
            engine = XgmiShardedLookup(evs, 1, 0, B, dev, dedup=args.dedup)
            engine_kind = "xgmi peer-write"
        elif want == "xgmi":
            # peer writes over xGMI; every rank must succeed or all fall back
            ok, err = 1, ""
            try:
                barrier = None
                if staged:
                    def barrier():
                        torch.cuda.synchronize()
                        dist.barrier()
                engine = XgmiShardedLookup(evs, world, rank, B, dev, barrier=barrier,
                                           dedup=args.dedup)
            except Exception as e:  # IPC mapping unavailable
                ok, err = 0, str(e)
            flag = torch.tensor([ok], dtype=torch.int32, device="cpu" if staged else dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if int(flag.item()) == 1:
                engine_kind = "xgmi peer-write"
            else:
                log("xgmi engine unavailable on some rank (%s); RCCL all-to-all engine" % err)
                if engine is not None:
                    engine.close()
                engine = None
        a2a = ShardedLookup(evs, world, rank, B, dev)
        if staged:
            def staged_a2a(out, inp, out_splits=None, in_splits=None):
                o = torch.empty(out.shape, dtype=out.dtype)
                dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
                out.copy_(o)
                return out
            a2a._a2a = staged_a2a
        elif world == 1:
            a2a._a2a = lambda out, inp, os_=None, is_=None: out.copy_(inp)
        if engine is None:
            engine = a2a
            engine_kind = "RCCL all-to-all"
        if args.dedup and engine is not None and engine is not a2a:
            engine_kind += " + dedup"
        log("sharded engine: %s" % engine_kind)
    else:
        engine = None
        keyspace = R
    batches = make_batches(4, T, B, keyspace, args.zipf, 2021 + 7919 * rank, dev)
    engine_check = None
    phases = None

    def engines_agree(steps):
        """The peer-write engine must reproduce the all-to-all engine bit for
        bit: compared on the given batch indices, with the output consumed
        (read) between steps, and-reduced over ranks."""
        same = 1
        with torch.no_grad():
            for k in steps:
                got = engine.forward(batches[k]).clone()
                float(got.sum())                      # consume, as a model step would
                same &= int(torch.equal(got, a2a.forward(batches[k])))
        if world > 1:
            flag = torch.tensor([same], dtype=torch.int32, device="cpu" if staged else dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            same = int(flag.item())
        return bool(same)

    if engine is not None and engine is not a2a:
        ok0 = engines_agree([0, 1, 2, 3])
        engine_check = "xgmi == all-to-all output, steps 0-3, all ranks: %s" % ok0
        log(engine_check)
        if not ok0:
            engine.close()
            engine, engine_kind = a2a, "RCCL all-to-all (xgmi check failed)"
    seg = torch.arange(B, dtype=torch.int32, device=dev)
    ind = torch.stack([torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64, device=dev)], 1)
    static_ids = torch.empty((T, B), dtype=torch.int64, device=dev)
    # the id batches are resident in HBM (value counts no host->device input
    # traffic); step k reads batch k % 4 in place.  At N = 1 a batch is a
    # record-major [B, T] id matrix (one Criteo record of T categorical ids
    # per row, the SOK/DLRM Criteo-TB input) whose columns are the features'
    # SparseTensor values: the fused lookup reads it in place
    # (dr_ev_lookup_onehot_strided).  The training step and the sharded
    # engines take the feature-major [T, B] form.
    recs = [ids.t().contiguous() for ids in batches]
    batch_sps = [[SparseTensor(ind, ids[t], (B, 1)) for t in range(T)] for ids in batches]
    rec_sps = [[SparseTensor(ind, r[:, t], (B, 1)) for t in range(T)] for r in recs]

    def step(k):
        if engine is not None:
            return engine.forward(batches[k])
        return dr.embedding_lookup_sparse_multi(evs, rec_sps[k], combiner="sum")

    NBATCH = len(batches)
    torch.cuda.synchronize()
    with torch.no_grad():
        for w in range(max(args.warmup, 2)):
            out = step(w % NBATCH)
            torch.cuda.synchronize()
            log("eager warmup step %d ok" % w)
        dr.status_check(dev)
        graph_all = None
        if not args.no_graph and engine is None:
            # one graph of the NBATCH steps in a row (a graph launch costs
            # ~10 us between replays; hipGraph-captured inner loop with every
            # step's full work inside); leftover steps run eagerly
            graph_all = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph_all):
                for k in range(NBATCH):
                    out = step(k)
            log("graphs captured")
            graph_all.replay()
            torch.cuda.synchronize()
            log("graph replay ok")

        debug = os.environ.get("DR_BENCH_DEBUG") == "1"

        def run_steps(i0, n):
            i = i0
            while i < i0 + n:
                if graph_all is not None and i % NBATCH == 0 and i + NBATCH <= i0 + n:
                    graph_all.replay()
                    i += NBATCH
                    continue
                step(i % NBATCH)
                if debug:
                    torch.cuda.synchronize()
                    log("step %d: done" % i)
                i += 1

        # N > 1 peer-write engine: HIP events between its phases during the
        # timed steps (route / barrier / serve / barrier; phase_summary)
        phase_engine = (engine if engine is not None and hasattr(engine, "phase_timing")
                        and not getattr(engine, "dedup", False) and world > 1 else None)

        def timed():
            run_steps(0, args.warmup)
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            if phase_engine is not None:
                phase_engine.phase_timing(True)
            t0 = time.perf_counter()
            run_steps(0, args.steps)
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            return time.perf_counter() - t0

        el = timed()
        log("timed %d steps in %.3fs" % (args.steps, el))
        phases = None
        if phase_engine is not None:
            phases = exchange_phases(phase_engine.phase_summary(), batches, world, rank, T, D,
                                     dist, staged, dev)
            phase_engine.phase_timing(False)
            log("exchange phases: %s" % json.dumps(phases))
        if engine is not None and engine is not a2a:
            # the last timed step's output (still in the engine's buffer),
            # then two more steps, against the all-to-all engine
            with torch.no_grad():
                kl = (args.steps - 1) % NBATCH
                last = (engine.forward(batches[kl]) if engine.dedup else engine.bufs.out).clone()
                same = int(torch.equal(last, a2a.forward(batches[kl])))
                if world > 1:
                    flag = torch.tensor([same], dtype=torch.int32,
                                        device="cpu" if staged else dev)
                    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
                    same = int(flag.item())
            ok1 = bool(same) and engines_agree([(kl + 1) % NBATCH, (kl + 2) % NBATCH])
            engine_check += "; last timed step + 2 more after timing: %s" % ok1
            log(engine_check)
            if not ok1:
                engine.close()
                engine, engine_kind = a2a, "RCCL all-to-all (xgmi check failed after timing)"
                el = timed()
                log("re-timed with the all-to-all engine: %.3fs" % el)
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device="cpu" if staged else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # the library's own sharded C entries (dr_sharded_forward over a dr_comm:
    # RCCL, ncclUniqueId through torch.distributed; N = 1 too, where every
    # all-to-all is the self block inside an RCCL group) beside the headline
    native = None
    if args.native_steps > 0:
        try:
            native = native_rccl_leg(args, evs, batches, engine, a2a if engine is not None else None,
                                     step, world, rank, dist, staged, dev, log)
        except Exception as e:  # noqa: BLE001 -- an extra leg must not cost the headline line
            log("native RCCL leg failed: %r" % (e,))
            native = {"error": str(e)[:300]}
    lookups = T * B * args.steps * world
    value = lookups / el
    ms = el / args.steps * 1e3
    dr.status_check(dev)

    # ---- parity at the headline size, outside the timed region: sampled
    # output rows == the tables' synth rows bit for bit (every key exists);
    # N = 1 also runs a step with ~10 % new keys (insert-on-miss: default
    # rows, EV sizes grow by the distinct new keys) and a Zipf(1.05) step
    correctness = {"checked_rows": 0}
    with torch.no_grad():
        kc = (args.steps - 1) % NBATCH
        outc = step(kc)
        correctness["checked_rows"] += check_rows(outc, batches[kc], T, D, args.check_rows,
                                                  17 + rank)
        if world == 1 and engine is None:
            gz = torch.Generator(device=dev)
            gz.manual_seed(99)
            ids = torch.randint(0, R, (T, B), generator=gz, device=dev, dtype=torch.int64)
            newm = torch.rand((T, B), generator=gz, device=dev) < 0.1
            ids = torch.where(newm, R + torch.randint(0, 1 << 40, (T, B), generator=gz,
                                                      device=dev, dtype=torch.int64), ids)
            before = [int(ev.total_count()[0]) for ev in evs]
            sps = [SparseTensor(ind, ids[t], (B, 1)) for t in range(T)]
            outn = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
            dr.status_check(dev)
            view = outn.view(B, T, D)
            old_ok = ~newm.t()                          # [B, T]
            for t in range(T):
                added = int(evs[t].total_count()[0]) - before[t]
                want = int(torch.unique(ids[t][newm[t]]).numel())
                if added != want:
                    raise AssertionError("table %d grew by %d keys, expected %d" % (t, added, want))
            if bool((view[~old_ok] != 0).any()):
                raise AssertionError("new keys must read the EV default row (0)")
            keep = torch.nonzero(old_ok.t().reshape(-1)).reshape(-1)[:args.check_rows]
            tb = keep // B
            bb = keep % B
            got = view[bb, tb].cpu().numpy()
            kk = ids[tb, bb].cpu().numpy()
            tt = tb.cpu().numpy()
            for t in np.unique(tt):
                if not np.array_equal(got[tt == t], synth_rows(1000 + int(t), kk[tt == t], D)):
                    raise AssertionError("new-key step: existing rows differ (table %d)" % t)
            correctness["checked_rows"] += int(keep.numel())
            correctness["new_key_step"] = {"new_keys": int(newm.sum()),
                                           "ev_growth_exact": True,
                                           "defaults_for_new": True}
            zk = (torch.as_tensor(np.random.default_rng(5).zipf(1.05, size=(T, B)),
                                  device=dev) - 1) % R
            zsp = [SparseTensor(ind, zk[t], (B, 1)) for t in range(T)]
            outz = dr.embedding_lookup_sparse_multi(evs, zsp, combiner="sum")
            correctness["checked_rows"] += check_rows(outz, zk, T, D, args.check_rows, 23)
            correctness["zipf_step"] = {"alpha": 1.05, "distinct_keys_table0":
                                        int(torch.unique(zk[0]).numel())}
        dr.status_check(dev)
    correctness["bitexact"] = True
    correctness["status"] = "clean"
    log("headline-size parity: %s" % json.dumps(correctness))

    # ---- embedding training step (N = 1): forward (grouped Unique -> EV
    # resolve -> pool) + backward (grouped segment grad) + KV SGD apply
    train = None
    if world == 1 and engine is None and args.train_steps > 0:
        opt = dr.GradientDescentOptimizer(0.01)
        upstream = torch.randn((B, T * D), device=dev)

        def tstep(i):
            out = dr.embedding_lookup_sparse_multi(evs, batch_sps[i % NBATCH], combiner="sum")
            out.backward(upstream)
            opt.apply_gradients(evs)

        for i in range(2):
            tstep(i)
        torch.cuda.synchronize()
        tgraph = None
        if not args.no_graph:
            # NBATCH whole training steps (forward, autograd backward, KV
            # apply) captured as one hipGraph: every kernel of every step runs
            # on replay, only the host's per-launch work is gone
            for ev in evs:   # worst-case adds of the captured steps (resolve + apply)
                ev.reserve(2 * NBATCH * B)
            tgraph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(tgraph):
                for i in range(NBATCH):
                    tstep(i)
            tgraph.replay()
            torch.cuda.synchronize()
            dr.status_check(dev)
        nsteps = args.train_steps
        t0 = time.perf_counter()
        if tgraph is not None:
            nsteps = -(-nsteps // NBATCH) * NBATCH
            for i in range(0, nsteps, NBATCH):
                tgraph.replay()
        else:
            for i in range(nsteps):
                tstep(i)
        torch.cuda.synchronize()
        tel = time.perf_counter() - t0
        dr.status_check(dev)
        tms = tel / nsteps * 1e3
        train = {"ms_per_step": round(tms, 4), "samples_per_s": round(B / (tms * 1e-3), 1),
                 "lookups_per_s": round(T * B / (tms * 1e-3), 1), "steps": nsteps,
                 "graph": tgraph is not None,
                 "step": "embedding layer training step: embedding_lookup_sparse_multi forward "
                         "(fused EV probe + row copy recording each id's row) + backward (row-grouped "
                         "segment grad) fused with the KV SGD update "
                         "(dr_ev_pool_grad_rows_apply_sgd), %d EVs, B=%d" % (T, B)}
        log("train step: %s" % json.dumps(train))
    elif world > 1 and engine is not None and args.train_steps > 0:
        # ---- embedding training step at N > 1: sharded forward (ids to
        # their owners, owner resolve, rows back), sharded backward (the
        # owners pull / receive their keys' gradient rows -> IndexedSlices on
        # their EV shards), owner KV SGD apply.  Eager (the exchange's
        # barriers are stream-ordered collectives); every rank's own batch.
        opt = dr.GradientDescentOptimizer(0.01)
        gu_ = torch.Generator(device=dev)
        gu_.manual_seed(77 + rank)
        upstream = torch.randn((B, T * D), generator=gu_, device=dev)

        def tstep(i):
            ids = batches[i % NBATCH]
            if engine is a2a:
                engine.forward(ids, need_grad=True)
            else:
                engine.forward(ids)
            engine.backward(upstream)
            opt.apply_gradients(evs)

        for i in range(2):
            tstep(i)
        torch.cuda.synchronize()
        dr.status_check(dev)
        nsteps = args.train_steps
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nsteps):
            tstep(i)
        dist.barrier()
        torch.cuda.synchronize()
        tel = time.perf_counter() - t0
        te = torch.tensor([tel], dtype=torch.float64, device="cpu" if staged else dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        tel = float(te.item())
        dr.status_check(dev)
        tms = tel / nsteps * 1e3
        train = {"ms_per_step": round(tms, 4),
                 "samples_per_s": round(world * B / (tms * 1e-3), 1),
                 "lookups_per_s": round(world * T * B / (tms * 1e-3), 1), "steps": nsteps,
                 "graph": False, "engine": engine_kind,
                 "step": "sharded embedding layer training step: forward (%s exchange) + "
                         "backward to the owners (IndexedSlices on their EV shards) + owner KV "
                         "SGD apply, %d EVs, B_local=%d, global batch %d"
                         % (engine_kind, T, B, world * B)}
        log("train step: %s" % json.dumps(train))

    # ---- DLRM model training step on the headline tables (modelzoo.DLRM,
    # bf16 MFMA towers): at N > 1 data-parallel with the row-sharded lookup
    # (train_step_sharded: dense gradients all-reduced, embedding gradient
    # rows to their owners), at N = 1 the local lookup.  Eager, barrier-
    # bracketed, max over ranks; samples/s over the global batch.
    dlrm = None
    if args.model_steps > 0:
        from deeprec_amd import modelzoo as mz
        torch.manual_seed(0)
        sharded_model = world > 1 and engine is not None
        model = mz.DLRM(evs, 13, bf16=True, engine=engine if sharded_model else None).to(dev)
        dopt = torch.optim.SGD(model.parameters(), lr=0.01)
        eopt = dr.GradientDescentOptimizer(0.01)
        gd = torch.Generator(device=dev)
        gd.manual_seed(5 + rank)
        mdense = [torch.randn((B, 13), generator=gd, device=dev) for _ in range(NBATCH)]
        mlab = [(torch.rand(B, generator=gd, device=dev) > 0.5).float() for _ in range(NBATCH)]

        def mstep(i):
            k = i % NBATCH
            if sharded_model:
                return mz.train_step_sharded(model, mdense[k], batches[k], mlab[k], dopt, eopt,
                                             world, staged=staged)
            return mz.train_step(model, mdense[k], batches[k], mlab[k], dopt, eopt)

        for i in range(2):
            mstep(i)
        torch.cuda.synchronize()
        dr.status_check(dev)
        # N = 1: NBATCH whole model steps (forward, backward, dense SGD, KV
        # SGD) captured as one hipGraph, as the embedding training step; the
        # eager loop if anything in the step refuses capture
        # Before it is timed, the graph is checked against the eager steps
        # from the same state (parameters and every touched EV row saved and
        # restored; SGD keeps no other state), replayed twice with eager work
        # between: any bit that differs and the eager loop is timed instead
        mgraph, mcheck, mlosses = None, None, None
        if not sharded_model and not args.no_graph and args.model_graph:
            try:
                for ev in evs:
                    ev.reserve(2 * NBATCH * B)
                mgraph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(mgraph):
                    mlosses = [mstep(i) for i in range(NBATCH)]
                mcheck = _dlrm_graph_check(mgraph, mlosses, mstep, model, evs,
                                           [batches[k] for k in range(NBATCH)], D, NBATCH)
                dr.status_check(dev)
                if not mcheck.startswith("equal"):
                    log("dlrm model step: graph check failed (%s); eager" % mcheck)
                    mgraph = None
            except Exception as e:  # noqa: BLE001
                log("dlrm model step: graph capture failed (%s); eager" % str(e)[:200])
                mgraph = None
                torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        nsteps = args.model_steps
        t0 = time.perf_counter()
        if mgraph is not None:
            nsteps = -(-nsteps // NBATCH) * NBATCH
            for i in range(0, nsteps, NBATCH):
                mgraph.replay()
        else:
            for i in range(nsteps):
                mstep(i)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        mel = time.perf_counter() - t0
        if dist is not None:
            te = torch.tensor([mel], dtype=torch.float64, device="cpu" if staged else dev)
            dist.all_reduce(te, op=dist.ReduceOp.MAX)
            mel = float(te.item())
        dr.status_check(dev)
        mms = mel / nsteps * 1e3
        dlrm = {"ms_per_step": round(mms, 4),
                "samples_per_s": round(world * B / (mms * 1e-3), 1),
                "global_batch": world * B, "steps": nsteps, "graph": mgraph is not None,
                "graph_check": mcheck,
                "engine": engine_kind if sharded_model else "local",
                "model": "modelzoo/DLRM/train.py DLRM, dot interaction, bf16 MFMA towers: bottom "
                         "[13, 512, 256, %d], top [%d, 512, 256] + 1-unit output, BCE; SGD on "
                         "the dense weights%s, KV SGD on the %d EV%s" % (
                             D, D + (T + 1) * T // 2,
                             " (all-reduced gradients)" if sharded_model else "", T,
                             " shards" if sharded_model else "s")}
        log("dlrm model step: %s" % json.dumps(dlrm))
        # (the captured losses live in the graph's private pool: drop them too)
        model = dopt = eopt = mdense = mlab = mgraph = mlosses = None
    din = None
    if args.din_steps > 0:
        try:
            din = din_leg(args, dev, log, world, rank, dist, staged)
        except Exception as e:  # noqa: BLE001 -- an extra leg must not cost the headline line
            log("din leg failed: %r" % (e,))
            din = {"error": str(e)[:300]}

    # ---- dominant kernel: the fused one-hot EV lookup, timed alone --------
    # dr_ev_lookup_onehot on keys this rank owns (all keys at N=1), over the
    # timed region's four step batches in rotation (a batch repeated launch
    # after launch finds part of its rows still in the Infinity Cache and
    # reads ~8 % faster than the steps do).  dr_kernel_timing brackets every
    # launch of the probe + row-copy kernel itself with HIP events on its
    # stream: the id concat and the three miss-list kernels (empty here) are
    # outside the bracket.
    import ctypes as _C
    from deeprec_amd.embedding_ops import _Feature, _fused_onehot
    L = _lib.lib()

    def kernel_ms(which, launch, n):
        L.dr_kernel_timing(which)
        for i in range(n):
            launch(i)
        torch.cuda.synchronize()
        tot, cnt = _C.c_double(0.0), _C.c_int64(0)
        _lib.check(L.dr_kernel_timing_result(_C.byref(tot), _C.byref(cnt)))
        L.dr_kernel_timing(0)
        if cnt.value != n:
            raise RuntimeError("kernel timing bracketed %d of %d launches" % (cnt.value, n))
        return tot.value / cnt.value

    own = [((batches[k] % R) * world + rank).contiguous() for k in range(len(batches))]
    own_rec = [o.t().contiguous() for o in own]           # record-major, as the steps
    with torch.no_grad():
        kfeats = [[_Feature(evs[t], own_rec[k][:, t], seg, B, None, "sum", None, onehot=True)
                   for t in range(T)] for k in range(len(own))]
        for fs in kfeats:
            assert _fused_onehot(fs, _lib.ORDER_ALI) is not None
        torch.cuda.synchronize()
        k_ms = kernel_ms(1, lambda i: _fused_onehot(kfeats[i % len(kfeats)], _lib.ORDER_ALI),
                         args.kernel_iters)
    log("lookup kernel %.4f ms/launch over %d launches on rotating batches"
        % (k_ms, args.kernel_iters))

    # ---- the north_star's row-gather target: the same
    # lookups on pre-resolved rows (dr_ev_resolve_grouped once per batch,
    # outside the timing), pool_onehot_kernel alone: 8 (row id) + D*4 read +
    # D*4 write, over the same rotating batches
    from deeprec_amd.embedding_ops import _pool_all, _prepare_group
    with torch.no_grad():
        gsets = []
        for k in range(len(own)):
            gfeats = [_Feature(evs[t], own[k][t], seg, B, None, "sum", None, onehot=True)
                      for t in range(T)]
            _prepare_group(gfeats, need_grad=False)
            _pool_all(gfeats, _lib.ORDER_ALI)
            gsets.append(gfeats)
        torch.cuda.synchronize()
        g_ms = kernel_ms(2, lambda i: _pool_all(gsets[i % len(gsets)], _lib.ORDER_ALI),
                         args.kernel_iters)
    g_per = 8 + 2 * D * 4
    g_ach = T * B * g_per / (g_ms * 1e-3) / 1e9
    roof_gather = {"bound": "hbm", "achieved": round(g_ach, 1), "peak": PEAK_HBM_GBS,
                   "unit": "GB/s", "frac": round(g_ach / PEAK_HBM_GBS, 4), "traffic": None,
                   "kernel": "dr::pool_onehot_kernel<4,32,1,ALI,4> on pre-resolved rows "
                             "(BASELINE.md row-gather target, >= 0.70)",
                   "kernel_ms": round(g_ms, 4), "bytes_per_launch": T * B * g_per,
                   "bytes_per_lookup": g_per}
    # SURVEY 8(d) EV hashed gather (+ the pooled write): key 8 + slot 16 +
    # row D*4 read + D*4 output write per lookup (h = 1)
    per_lookup = 8 + 16 + D * 4 + D * 4
    bytes_launch = T * B * per_lookup
    achieved = bytes_launch / (k_ms * 1e-3) / 1e9
    # which fused lookup kernel the library launches (DR_LOOKUP_KERNEL, ev.hip)
    lk_kind = os.environ.get("DR_LOOKUP_KERNEL", "1")
    lk_name = {"0": "ev_lookup_onehot_kernel", "1": "ev_lookup_line_kernel"}.get(
        lk_kind, "ev_lookup_pipe_kernel")
    lk_inst = {"0": "<4,32,1,ALI,4>"}.get(lk_kind, "<4,32,1,ALI>")
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
            "kernel": "dr::%s%s (record-major [B, T] ids)" % (lk_name, lk_inst),
            "kernel_ms": round(k_ms, 4),
            "bytes_per_launch": bytes_launch, "bytes_per_lookup": per_lookup}
    import glob as _glob

    def _latest(suffix):
        fs = sorted(_glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_" + suffix)))
        return fs[-1] if fs else None

    for obj, fname, kname in ((roof, _latest("pmc_traffic.json"), lk_name),
                              (roof_gather, _latest("pmc_traffic_row_gather.json"),
                               "pool_onehot_kernel")):
        if fname:
            try:
                j = json.load(open(fname))
                # PMC of this same kernel only (rocprof names the template
                # instantiation, e.g. "ev_lookup_onehot_kernel<4, 32, 1, 0, 4>")
                if str(j.get("kernel", "")).startswith(kname):
                    obj["traffic"] = j.get("bytes_per_launch")
                    obj["traffic_source"] = os.path.relpath(fname, ROOT)
                    # the profile's round and the instantiation it measured
                    obj["traffic_round"] = os.path.basename(fname)[:3]
                    obj["traffic_kernel"] = j.get("kernel")
            except Exception:
                pass

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args)

    deepfm = criteo = dcn = hybrid = None
    if (world == 1 and (args.deepfm or args.criteo or args.dcn)) or args.hybrid:
        # drop every holder of the headline EVs so their HBM is released;
        # each leg below frees its own tables before the next one
        # (loop variables too: `fs` holds a feature list of every table, `ev`
        # the last table -- either kept 180 GB of headline tables alive)
        evs = feats = gfeats = batch_sps = rec_sps = kfeats = gsets = fs = ev = None
        engine = a2a = outc = graph_all = tgraph = opt = step = tstep = mstep = None
        _free_hbm()
        log("HBM free after the headline tables: %.1f GB" % (torch.cuda.mem_get_info(dev)[0] / 1e9))
        if world == 1 and args.deepfm:
            deepfm = deepfm_leg(args, dev, log)
            _free_hbm()
        if world == 1 and args.criteo:
            criteo = criteo_legs(args, dev, log)
            _free_hbm()
        if world == 1 and args.dcn:
            dcn = dcn_bf16_leg(args, dev, log)
            _free_hbm()
        if args.hybrid:
            hybrid = criteo_hybrid_leg(args, dev, log, world, rank, dist, staged)
            _free_hbm()

    if rank == 0:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            metric = json.load(f)["metric"]
        line = {
            "metric": metric,
            "value": round(value, 1),
            "unit": "lookups/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (uniform keys%s, hash-derived table rows)" % (
                "" if args.zipf <= 0 else ", zipf %.2f" % args.zipf),
            "config": {"workload": "DLRM Criteo-TB shape: %d EV tables x %d rows/GPU x %d fp32, "
                                   "B_local=%d, hotness 1, embedding_lookup_sparse(sum) forward "
                                   "(EV insert-on-miss resolve of every id -> fused gather+pool; "
                                   "forward-only filter-free one-hot needs no Unique)%s"
                                   % (T, R, D, B, "; %s exchange: ids to owners (key %% N), "
                                      "owner resolve, rows back" % engine_kind
                                      if world > 1 else ""),
                       "global_batch": B * world, "tables": T, "rows_per_gpu": R, "dim": D,
                       "engine": engine_kind, "engine_check": engine_check,
                       "parallelism": "row-sharded tables x%d, data-parallel batch" % world},
            "forward_samples_per_s": round(value / T, 1),
            "train_step": train,
            "dlrm_train_step": dlrm,
            "din_config": din,
            "deepfm_config": deepfm,
            "criteo_tb_cardinalities": criteo,
            "criteo_tb_hybrid": hybrid,
            "exchange_phases": phases,
            "native_engine": native,
            "dcn_bf16_config": dcn,
            "correctness": correctness,
            "roofline": roof,
            "roofline_row_gather": roof_gather,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
