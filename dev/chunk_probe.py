"""Host cost of splitting a Trainer-managed parameter (flat-buffer view) with chunk vs slicing,
in grad mode -- the training forward's per-layer in_proj splits."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cmt-cooperative-perception_amd"))
from projects.mmdet3d_plugin import synthetic as S  # noqa: E402
from projects.mmdet3d_plugin.trainer import Trainer  # noqa: E402


def main():
    head, _, _ = S.build_synthetic_head("cmtcoop_fusion_tumtraf", seed=0, num_query=900, device="cuda")
    head.train()
    Trainer(head, lr=1e-4)
    w = head.transformer.decoder.layers[0].attentions[0].attn.in_proj_weight
    b = head.transformer.decoder.layers[0].attentions[0].attn.in_proj_bias
    C = w.shape[1]
    for name, fn in [("chunk", lambda: (w.chunk(3), b.chunk(3))),
                     ("slice", lambda: ((w[:C], w[C:2 * C], w[2 * C:]), (b[:C], b[C:2 * C], b[2 * C:]))),
                     ("split", lambda: (w.split(C), b.split(C)))]:
        for _ in range(10):
            fn()
        t0 = time.perf_counter()
        for _ in range(2000):
            fn()
        print(f"{name}: {(time.perf_counter() - t0) / 2000 * 1e6:.1f} us per weight+bias split", flush=True)


if __name__ == "__main__":
    main()
