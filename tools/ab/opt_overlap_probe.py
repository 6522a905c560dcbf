"""Round 6: can the optimizer step (grad norm + AdamW + the mapper's transposed copies, HBM-bound) hide under the next
step's CLIP-B/32 forward (GEMM-bound, independent of the optimizer)? HIP graphs of: the CLIP forward alone, the
optimizer alone, and both on two streams forked from one point; median of 20 replays each (ms)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-image-captioning_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from icap import ops  # noqa: E402


def timed(g, n=20):
    ts = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(n):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def main():
    dev = torch.device("cuda", 0)
    B = 128
    model, tower, tr = bench.build(B, dev)
    ids, mask, labels, px = bench.synthetic_batch(B, 1, dev)
    tr.load_batch(ids, mask, labels, pixels=px)
    for _ in range(2):
        tr.micro_step(use_graph=True)
    torch.cuda.synchronize()
    clip = lambda: tr.clip.run(tr.cws, tr.pixels)  # noqa: E731
    opt = tr._optimizer
    side = torch.cuda.Stream(dev)
    ops.register_side_stream(side)
    graphs = {}
    for name in ("clip", "opt", "both"):
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with ops.graph_capture(g):
            if name == "clip":
                clip()
            elif name == "opt":
                opt()
            else:
                main_s = torch.cuda.current_stream()
                side.wait_stream(main_s)
                with torch.cuda.stream(side):
                    opt()
                clip()
                main_s.wait_stream(side)
        graphs[name] = g
    for rep in range(2):
        r = {k: timed(g) for k, g in graphs.items()}
        print(f"clip {r['clip']:.3f} ms  opt {r['opt']:.3f} ms  sum {r['clip'] + r['opt']:.3f}  both {r['both']:.3f}  "
              f"saved {r['clip'] + r['opt'] - r['both']:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
