"""Pure-torch check of the capture pattern tools/din_graph_probe.py uses:
an MLP step (forward, loss, zero_grad(set_to_none), backward, capturable
Adam) captured as two graphs over two batches and replayed alternately,
against the same steps eagerly -- with zero_grad inside the captured step
(as modelzoo.din_train_step) and, the documented pattern, before each
capture."""
import torch


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    xs = [torch.randn(512, 64, device=dev) for _ in range(2)]
    ys = [torch.randn(512, 1, device=dev) for _ in range(2)]

    def make():
        torch.manual_seed(1)
        m = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(),
                                torch.nn.Linear(128, 1)).to(dev)
        g = torch.nn.Parameter(torch.ones(128, device=dev))
        return m, g, torch.optim.Adam(list(m.parameters()) + [g], lr=1e-3, capturable=True)

    def step(m, g, opt, i, inner_zero):
        h = torch.relu(m[0](xs[i % 2])) * g
        loss = ((m[2](h) - ys[i % 2]) ** 2).mean()
        if inner_zero:
            opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for inner in (True, False):
        A, B = make(), make()
        for i in range(3):
            for M in (A, B):
                M[2].zero_grad(set_to_none=True)
                step(*M, i, True)
        graphs = []
        for j in range(2):
            if not inner:
                B[2].zero_grad(set_to_none=True)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                step(*B, 3 + j, inner)
            graphs.append(gr)
        ok = True
        for i in range(3, 9):
            A[2].zero_grad(set_to_none=True)
            step(*A, i, True)
            graphs[(i - 3) % 2].replay()
            torch.cuda.synchronize()
            pa = list(A[0].parameters()) + [A[1]]
            pb = list(B[0].parameters()) + [B[1]]
            same = all(torch.equal(a, b) for a, b in zip(pa, pb))
            if not same:
                print("zero_grad %s capture: step %d differs" % ("inside" if inner else "before",
                                                                   i), flush=True)
                ok = False
                break
        print("zero_grad %s capture: graphs == eager: %s" % ("inside" if inner else "before", ok),
              flush=True)


if __name__ == "__main__":
    main()
