"""Round 6: which part of the captured DIN step goes wrong when the caching
allocator is churned between replays (tools/graph_mem_probe.py: the second
replay's forward is NaN after 3000 small allocations filled with NaN or
zeros, while zero-poisoning every free block of every pool is harmless).

One graph of one batch (batch 0), replayed GPP_REPLAYS times; GPP_PIECE:
  lookup  the uid and item EV lookups only (sum of the outputs)
  attn    lookups + the fused attention (sum of its outputs)
  attn_mlp / attn_pool   lookups + only the fused MLP / only the pool kernel
  fwd     forward + loss only (no state change: every replay must equal the first)
  fwdbwd  + backward (EV gradients dropped)
  dense   + dense Adam
  ev      + KV Adam on the EVs (no dense update)
  full    the whole step
GPP_CHURN=1 churns the allocator before every replay (as graph_mem_probe's
"small"); GPP_CHURN_KIND=alloc: allocations without kernels, =launch:
3000 kernel launches without allocations.  The printed loss sequence of a churned run is diffed against the
unchurned run's (both deterministic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import din_graph_probe as dgp  # noqa: E402


def _hip():
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemsetD32Async.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
    return hip


def _fill(hip, blocks, word, dev):
    import ctypes as C
    st = torch.cuda.current_stream(dev).cuda_stream
    for a, sz in blocks:
        assert hip.hipMemsetD32Async(C.c_void_p(a), word, sz // 4, C.c_void_p(st)) == 0
    torch.cuda.synchronize()


def bisect(g, loss, dev):
    """GPP_BISECT=1: NaN-fill free blocks (of the default pool, or every
    pool with GPP_POOLS=all) and replay the captured piece; when that
    changes the output, halve the set (zero-filling each tried half
    afterwards) down to the one block the graph reads."""
    hip = _hip()
    snap = torch.cuda.memory._snapshot()
    allp = os.environ.get("GPP_POOLS", "default") == "all"
    blocks = []
    for seg in snap["segments"]:
        if not allp and tuple(seg.get("segment_pool_id", (0, 0))) != (0, 0):
            continue
        for b in seg["blocks"]:
            if b["state"] == "inactive":
                blocks.append((b["address"], b["size"]))
    nan = 0x7FC00000

    def trial(bs):
        _fill(hip, blocks, 0, dev)
        _fill(hip, bs, nan, dev)
        g.replay()
        torch.cuda.synchronize()
        return repr(float(loss.detach()))
    base = trial([])
    print("free blocks: %d (%d B); zero-filled replay: %s" % (
        len(blocks), sum(s for _, s in blocks), base), flush=True)
    cand = list(blocks)
    if trial(cand) == base:
        print("BISECT: NaN in every free block leaves the output unchanged", flush=True)
        return
    while len(cand) > 1:
        half = cand[:len(cand) // 2]
        cand = half if trial(half) != base else cand[len(cand) // 2:]
    a, sz = cand[0]
    print("BISECT: the graph reads the free block %#x (%d B)" % (a, sz), flush=True)
    for seg in snap["segments"]:
        if seg["address"] <= a < seg["address"] + seg["total_size"]:
            print("  segment %#x size %d pool %s stream %s" % (
                seg["address"], seg["total_size"], seg.get("segment_pool_id"), seg.get("stream")),
                flush=True)
    hist = snap.get("device_traces", [[]])[0]
    for e in hist:
        ea, es = e.get("addr"), e.get("size") or 0
        if ea is not None and ea <= a < ea + max(es, 1) and e.get("action") in (
                "alloc", "free_requested", "free_completed"):
            fr = [f for f in e.get("frames", []) if "site-packages/torch" not in f.get("filename", "")
                  or "optim" in f.get("filename", "")][:8]
            print("  %s %#x %d B: %s" % (e.get("action"), ea, es, " <- ".join(
                "%s:%s:%s" % (os.path.basename(f["filename"]), f["line"], f["name"]) for f in fr)),
                flush=True)


def const_piece(dr, dev, bt, piece):
    """const_pool: din_attention_pool on fixed facts / scores (no lookup),
    captured alone and replayed with the churn in between."""
    from deeprec_amd import ops as dops
    mask = bt[5]
    Bq, Tq = mask.shape
    g0 = torch.Generator(device=dev).manual_seed(3)
    facts = torch.randn(Bq, Tq, 36, generator=g0, device=dev)
    scores = torch.randn(Bq, Tq, generator=g0, device=dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        if piece == "const_pool":
            att, hs, _ = dops.din_attention_pool(scores, mask, facts)
        else:   # const_pool_sum: the scores from a torch reduction first
            att, hs, _ = dops.din_attention_pool(facts.sum(-1), mask, facts)
        loss = att.sum() + hs.sum()
    gen = torch.Generator().manual_seed(5)
    out = []
    for n in range(4):
        sizes = torch.randint(1, 1 << 18, (3000,), generator=gen).tolist()
        junk = [torch.full((s,), float("nan"), device=dev) for s in sizes]
        del junk
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        out.append(repr(float(loss)))
    print("LOSSES %s churn=1 %s" % (piece, " ".join(out)), flush=True)


def main():
    if os.environ.get("GPP_BISECT") == "1":
        torch.cuda.memory._record_memory_history(max_entries=2000000, stacks="python")
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    dr.load()
    dev = torch.device("cuda:0")
    B, T, D = int(os.environ.get("GPP_BATCH", "4096")), 100, 18
    R = (500_000, 400_000, 2_000)
    bat = dgp.batches_for(dev, B, T, R)
    piece = os.environ.get("GPP_PIECE", "full")
    evs, model, dopt, eopt = dgp.build(dr, mz, dev, "m", B, T, D, R)
    if piece.startswith("const_"):
        return const_piece(dr, dev, bat[0], piece)
    for i in range(4):
        mz.din_train_step(model, bat[i % 4], dopt, eopt, i)
    for ev in evs:
        ev.reserve(8 * B * (T + 1))
    torch.cuda.synchronize()
    bt = bat[0]

    def step():
        uids, mids, cats, mid_his, cat_his, mask, target = bt
        if piece in ("lookup", "attn", "attn_mlp", "attn_pool", "attn_pool_torch"):
            with torch.no_grad():
                Bq, Tq = mid_his.shape
                uid_e = model.uid_lookup(uids.reshape(1, Bq))
                ids = torch.stack([torch.cat([mids, mid_his.reshape(-1)]),
                                   torch.cat([cats, cat_his.reshape(-1)])])
                allv = model.item_lookup(ids)
                if piece == "lookup":
                    return allv.sum() + uid_e.sum()
                item_eb, facts = allv[:Bq], allv[Bq:].view(Bq, Tq, -1)
                m = model
                from deeprec_amd import ops as dops
                if piece == "attn_mlp":   # the fused MLP's kernels only
                    sc, _ = dops.din_mlp_forward(item_eb, facts, mask, m.f1_att.weight,
                                                 m.f1_att.bias, m.f2_att.weight, m.f2_att.bias,
                                                 m.f3_att.weight, m.f3_att.bias)
                    return sc.sum()
                if piece == "attn_pool":  # the pool kernel only (torch scores)
                    att, hs, _ = dops.din_attention_pool(facts.sum(-1), mask, facts)
                    return att.sum() + hs.sum()
                if piece == "attn_pool_torch":   # the same pool in torch ops
                    sc = torch.where(mask == 1, facts.sum(-1), torch.full_like(mask, -4294967296.0))
                    al = torch.softmax(sc, -1)
                    return (al[:, :, None] * facts).sum() + facts.sum()
                att, his_sum = mz.DinAttentionFused.apply(
                    item_eb, facts, mask, m.f1_att.weight, m.f1_att.bias, m.f2_att.weight,
                    m.f2_att.bias, m.f3_att.weight, m.f3_att.bias)
                return att.sum() + his_sum.sum()
        y = model(uids, mids, cats, mid_his, cat_his, mask)
        loss = -(torch.log(y) * target).mean()
        if piece == "fwd":
            return loss
        dopt.zero_grad(set_to_none=True)
        loss.backward()
        if piece in ("dense", "full"):
            dopt.step()
        if piece in ("ev", "full"):
            eopt.apply_gradients(model.evs, global_step=4)
        else:
            for ev in evs:
                ev.pending_grads = []
        return loss

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss = step()
    torch.cuda.synchronize()
    if os.environ.get("GPP_BISECT") == "1":
        return bisect(g, loss, dev)
    churn = os.environ.get("GPP_CHURN", "0") == "1"
    gen = torch.Generator().manual_seed(5)
    out = []
    for n in range(int(os.environ.get("GPP_REPLAYS", "4"))):
        if churn:
            kind = os.environ.get("GPP_CHURN_KIND", "fill")
            sizes = torch.randint(1, 1 << 18, (3000,), generator=gen).tolist()
            if kind == "fill":      # allocations + a fill kernel each
                junk = [torch.full((s,), float("nan"), device=dev) for s in sizes]
            elif kind == "alloc":   # allocations only, no kernel
                junk = [torch.empty((s,), device=dev) for s in sizes]
            else:                   # "launch": kernels only, on one buffer
                junk = torch.zeros(1 << 18, device=dev)
                for _ in sizes:
                    junk.add_(1.0)
            del junk
            torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        out.append(repr(float(loss.detach())))
        extra = ""
        if piece not in ("fwd", "lookup", "attn", "attn_mlp", "attn_pool", "attn_pool_torch"):
            bad = [nm for nm, p in model.named_parameters()
                   if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
            extra = " non-finite grads: %s" % (bad or "none")
        print("piece %s churn %d replay %d: loss %s%s" % (piece, churn, n, out[-1], extra),
              flush=True)
    print("LOSSES %s churn=%d %s" % (piece, churn, " ".join(out)), flush=True)


if __name__ == "__main__":
    main()
