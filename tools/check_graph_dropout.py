"""Does F.dropout inside a captured CUDA graph draw fresh masks on every replay (PyTorch's graph-safe
philox offsets)?  The independent-mask accuracy runs (tools/accuracy_parity.py, run_reference_graphed)
rely on it.  Prints the fraction of mask elements that differ between two replays and between a
replay and the eager call before capture; also checks the keep rate."""
import torch
import torch.nn.functional as F


def main():
    dev = torch.device("cuda:0")
    x = torch.ones(64, 16, 1, 64, device=dev)
    out = torch.empty_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            out.copy_(F.dropout(x, 0.25, training=True))
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out.copy_(F.dropout(x, 0.25, training=True))
    masks = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        masks.append((out != 0).clone())
    d01 = (masks[0] != masks[1]).float().mean().item()
    d12 = (masks[1] != masks[2]).float().mean().item()
    keep = torch.stack(masks).float().mean().item()
    print(f"replay-to-replay mask difference {d01:.3f} / {d12:.3f} (0 = frozen masks; ~0.375 = fresh), keep rate {keep:.3f}")


if __name__ == "__main__":
    main()
