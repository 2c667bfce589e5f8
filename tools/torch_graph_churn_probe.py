"""Round 6: does a graph of plain torch ops go wrong under the allocator
churn that breaks the captured DIN pieces (tools/graph_piece_probe.py
const_pool / attn_pool_torch)?  No deeprec_amd import unless --with-lib.

Pieces (TCP_PIECE): sum (x.sum()), softmax (masked softmax + weighted sum,
the DIN pool in torch ops), two_sums (a.sum() + b.sum()).  Fixed inputs,
one graph, replayed 4 times, 3000 NaN-filled tensors of 1 B - 1 MB
allocated and freed before each replay; every replay must give the first
replay's value."""
import os
import sys

import torch


def main():
    if "--with-lib" in sys.argv:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
            os.path.abspath(__file__))), "deeprec-1_amd"))
        import deeprec_amd as dr
        dr.load()
    dev = torch.device("cuda:0")
    piece = os.environ.get("TCP_PIECE", "softmax")
    B, T, H = 4096, 100, 36
    g0 = torch.Generator(device=dev).manual_seed(3)
    facts = torch.randn(B, T, H, generator=g0, device=dev)
    scores = torch.randn(B, T, generator=g0, device=dev)
    lens = torch.randint(1, T + 1, (B,), generator=g0, device=dev)
    mask = (torch.arange(T, device=dev)[None, :] < lens[:, None]).float()
    att = torch.randn(B, H, generator=g0, device=dev)
    torch.cuda.synchronize()

    def body():
        if piece == "sum":
            return facts.sum()
        if piece == "two_sums":
            return att.sum() + facts.sum()
        sc = torch.where(mask == 1, scores, torch.full_like(mask, -4294967296.0))
        al = torch.softmax(sc, -1)
        return (al[:, :, None] * facts).sum() + facts.sum()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss = body()
    gen = torch.Generator().manual_seed(5)
    out = []
    churn = os.environ.get("TCP_CHURN", "1") == "1"
    for _ in range(4):
        if churn:
            sizes = torch.randint(1, 1 << 18, (3000,), generator=gen).tolist()
            junk = [torch.full((n,), float("nan"), device=dev) for n in sizes]
            del junk
            torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        out.append(repr(float(loss)))
    print("TORCH %s lib=%d churn=%d %s -> %s" % (piece, "--with-lib" in sys.argv, churn,
                                                  " ".join(out),
                                                  "stable" if len(set(out)) == 1 else "CHANGES"),
          flush=True)


if __name__ == "__main__":
    main()
