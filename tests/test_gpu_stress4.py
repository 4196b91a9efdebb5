"""BASELINE.json configs[4], the 4-agent CMTCoop stress shape: 4 agents x
(LiDAR BEV + 4 cameras), 1500 queries, fp16 policy.

  * reduced size (32x32 BEV, 4 x 8x20 image maps per agent, 2 layers, 1500
    queries): 'ref' policy vs the oracle's 4-agent max fusion at the logit
    level (<= 1e-3 abs), and the fp16 policy vs the same oracle (<= 1 % of
    each output's scale);
  * full size (4 x 48 400 tokens, 6 layers, 1500 queries): 'ref' vs the
    oracle's 4-agent max fusion at the logit level (every layer, <= 1e-3 abs,
    headroom per key in the parity log) and the fp16 policy vs the same oracle
    (<= 1 % of each output's scale); and properties that hold exactly at fp16 --
    agent order does not change the max-fused outputs, and four copies of one
    agent equal that agent alone.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("center", "height", "dim", "rot", "vel", "cls_logits")
YAWS = (0.0, 90.0, 180.0, -90.0)


def _agents(n, hw, img_hw, seed):
    from projects.mmdet3d_plugin import synthetic as S
    agents, metas = [], {}
    for i in range(n):
        p = f"agent{i}_"
        x = S.synthetic_bev(1, hw, hw, seed=seed + 10 * i)
        xi = S.synthetic_img(len(YAWS), img_hw[0], img_hw[1], seed=seed + 10 * i + 1)
        pad = (img_hw[0] * 16, img_hw[1] * 16, 3)
        metas.update(S.synthetic_metas(1, yaws=YAWS, prefix=p, pad_shape=pad, seed=seed + 10 * i + 2)[0])
        agents.append((p, x, xi))
    return agents, [metas]


def _fwd(head, dev, prec, agents, metas):
    from projects.mmdet3d_plugin import set_precision
    set_precision(prec)
    try:
        with torch.no_grad():
            out = head.forward_agents([(p, x.to(dev), xi.to(dev)) for p, x, xi in agents], metas)[0]
        torch.cuda.synchronize()
    finally:
        set_precision("ref")
    return {k: v.cpu() for k, v in out.items()}


def test_stress4_reduced_parity(dev, parity_log):
    from oracle import cmt_oracle as O
    from projects.mmdet3d_plugin import synthetic as S
    head, cfg, _ = S.build_synthetic_head("cmtcoop_fusion_tumtraf", seed=0, num_query=1500, num_layers=2,
                                          grid_size=[256, 256, 40])
    oc, sd = O.cfg_from_head_cfg(cfg), S.head_state_dict(head)
    agents, metas = _agents(4, 32, (8, 20), seed=60)
    ref = O.head_coop_forward(oc, sd, agents, metas, "fusion", cross_core="fp16", epilogue=False)[0]
    head.to(dev)
    head.box_epilogue = False
    got = _fwd(head, dev, "ref", agents, metas)
    e = {k: (got[k].double() - ref[k].double()).abs().max().item() for k in KEYS}
    got16 = _fwd(head, dev, "fp16", agents, metas)
    r16 = {k: (got16[k].double() - ref[k].double()).abs().max().item() / max(ref[k].abs().max().item(), 1e-6)
           for k in KEYS}
    parity_log.append(f"stress4 reduced (4 agents, Nq 1500, L 2) 'ref' logits max abs {max(e.values()):.2e} "
                      f"bound 1e-3; 'fp16' max rel-to-scale {max(r16.values()):.2e} bound 1e-2")
    assert max(e.values()) <= 1e-3, e
    assert max(r16.values()) <= 1e-2, r16


def test_stress4_fullsize_parity(dev, parity_log):
    """configs[4] at full size against the oracle (cmt_head_coop.py:372-389, the max over
    agents generalised to four): 4 x (180 x 180 BEV + 4 x 40 x 100 camera tokens) = 4 x 48 400
    keys, 1500 queries, 6 layers."""
    from oracle import cmt_oracle as O
    from projects.mmdet3d_plugin import synthetic as S
    head, cfg, _ = S.build_synthetic_head("cmtcoop_fusion_tumtraf", seed=0, num_query=1500)
    oc, sd = O.cfg_from_head_cfg(cfg), S.head_state_dict(head)
    agents, metas = _agents(4, 180, (40, 100), seed=80)
    ref = O.head_coop_forward(oc, sd, agents, metas, "fusion", cross_core="fp16", epilogue=False)[0]
    head.to(dev)
    head.box_epilogue = False
    got = _fwd(head, dev, "ref", agents, metas)
    e = {k: (got[k].double() - ref[k].double()).abs().max().item() for k in KEYS}
    got16 = _fwd(head, dev, "fp16", agents, metas)
    r16 = {k: (got16[k].double() - ref[k].double()).abs().max().item() / max(ref[k].abs().max().item(), 1e-6)
           for k in KEYS}
    worst = max(e.values())
    parity_log.append(f"stress4 full size (4 x 48400 tokens, Nq 1500, L 6) 'ref' vs fp16-core oracle (logits): "
                      f"max abs {worst:.2e} (worst key {max(e, key=e.get)}, headroom {1 - worst / 1e-3:.0%}) "
                      f"[{', '.join(f'{k} {v:.1e}' for k, v in e.items())}] bound 1e-3; "
                      f"'fp16' max rel-to-scale {max(r16.values()):.2e} bound 1e-2")
    for k in KEYS:
        assert got[k].shape == ref[k].shape == (6, 1, 1500, ref[k].shape[-1]), k
    assert worst <= 1e-3, e
    assert max(r16.values()) <= 1e-2, r16


def test_stress4_fullsize_properties(dev, parity_log):
    from projects.mmdet3d_plugin import synthetic as S
    head, cfg, _ = S.build_synthetic_head("cmtcoop_fusion_tumtraf", seed=0, num_query=1500, device=dev)
    agents, metas = _agents(4, 180, (40, 100), seed=70)
    base = _fwd(head, dev, "fp16", agents, metas)
    perm = [agents[i] for i in (2, 0, 3, 1)]
    # the meta prefixes travel with their agents, so the permuted call sees the same (agent, camera) pairs
    rot = _fwd(head, dev, "fp16", perm, metas)
    for k in KEYS:
        assert torch.isfinite(base[k]).all(), k
        assert base[k].shape[:3] == (6, 1, 1500)
        assert torch.equal(base[k], rot[k]), k
    one = _fwd(head, dev, "fp16", agents[:1], metas)
    same = _fwd(head, dev, "fp16", [agents[0]] + [(f"agent{i}_", agents[0][1], agents[0][2]) for i in (1, 2, 3)],
                [{**metas[0], **{k.replace("agent0_", f"agent{i}_"): v for k, v in metas[0].items()
                                 if k.startswith("agent0_") for i in (1, 2, 3)}}])
    for k in KEYS:
        assert torch.equal(one[k], same[k]), k
    parity_log.append("stress4 full size (4 x 48400 tokens, Nq 1500, L 6, fp16): agent-order invariance and "
                      "4 identical agents == 1 agent hold bit-exactly")
