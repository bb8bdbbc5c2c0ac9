"""Where the fp8 recipe's loss spikes come from: the Llama-shape parity run (tests/test_training_parity_gpu.py, 2
layers, d_model 2048, GQA 32:4, 150 steps) in bf16 and in fp8 with per-step traces of every scale slot.

For each step and slot the trace holds the step's amax and the scale its casts used; ``r = amax * scale / FMAX`` > 1
means the cast saturated (values clipped to +-FMAX, the largest by a factor r).  The probe prints, per run, the
per-step loss gap to bf16 and, at the steps where the gap is largest, the slots that saturated.

    python benchmarks/fp8_spike_probe.py [--margins 1,2] [--history 16] [--out profiles/parity/fp8_spike_probe.json]

Slots (ops/fp8.py, models/transformer.py enable_fp8): e4m3 per layer 0 h1 (QKV input), 1 o (Wo input), 2 h2 (W13
input), 3 a (W2 input), 4-7 the weights (qkv, o, w13, w2); e5m2 per layer 0 dQKV, 1 dY of Wo, 2 dgu, 3 dY of W2.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests import test_training_parity_gpu as P  # noqa: E402

E4 = ["h1", "o", "h2", "a", "w_qkv", "w_o", "w_13", "w_2"]
E5 = ["dqkv", "dy_o", "dgu", "dy_2"]


def run(c, fp8: bool, margin: float, history: int, wgrad: bool, dev):
    from bpe_transformer.ops import gemm

    gemm._AUTOTUNE = False
    gemm._route.clear()
    ids, vocab = P._tokens()
    model = P._ours(vocab, c, dev)
    states = []
    if fp8:
        model.enable_fp8(history=history, margin=margin, wgrad=wgrad)
        states = model.fp8_states()
        for st in states:
            st.trace = []
    eng = P._engine(model, 1, c)
    data = P._batches(ids, P.STEPS, c.B, c.S, dev)
    losses = [eng.train_step([data[it]], lr=P._lr(it, c)) for it in range(P.STEPS)]
    losses = [float(v) for v in torch.stack(losses).cpu()]
    traces = []
    for st, names, fmax in zip(states, (E4, E5), (448.0, 57344.0)):
        t = torch.stack(st.trace).cpu()  # [steps, 2, n]
        ratio = (t[:, 0] * t[:, 1] / fmax).tolist()  # [steps][n]
        traces.append({"fmt": st.fmt, "names": names, "ratio": ratio, "amax": t[:, 0].tolist()})
    return losses, traces


def same_weights(c, steps, dev, margin=1.0):
    """Separate the fp8 forward's rounding from trajectory divergence: train bf16 and, before the bf16 step s, evaluate
    batch s on the SAME weights in bf16 and in fp8 -- with scales calibrated on the 16 preceding batches (what the
    delayed recipe would hold) and on batch s itself (just-in-time scaling)."""
    from bpe_transformer.ops import gemm

    gemm._AUTOTUNE = False
    gemm._route.clear()
    ids, vocab = P._tokens()
    model = P._ours(vocab, c, dev)
    eng = P._engine(model, 1, c)
    data = P._batches(ids, P.STEPS, c.B, c.S, dev)
    out = {}
    for it in range(max(steps) + 1):
        if it in steps:
            with torch.no_grad():
                x, y = data[it]
                lb = float(model.loss(x, y))
                model.enable_fp8(margin=margin)
                for jt in range(max(0, it - 16), it):
                    model.loss(*data[jt])
                    for st in model.fp8_states():
                        st.update()
                ld = float(model.loss(x, y))
                for st in model.fp8_states():
                    st.update()
                lj = float(model.loss(x, y))
                for layer in model.layers:
                    layer.fp8 = None
                model.fp8_state = model.fp8_grad_state = None
            out[it] = {"bf16": lb, "fp8_delayed": ld, "fp8_jit": lj, "rel_delayed": (ld - lb) / lb,
                       "rel_jit": (lj - lb) / lb}
            print(json.dumps({"same_weights_step": it, **{k: round(v, 4) for k, v in out[it].items()}}), flush=True)
        eng.train_step([data[it]], lr=P._lr(it, c))
    return out


def cross(c, steps, dev):
    """The other half of the split: train in fp8 and, before step s, evaluate batch s on the fp8-trained weights in
    fp8 and with fp8 switched off (bf16).  A spike that the bf16 evaluation of the same weights shows too is in the
    weights (the fp8 trajectory), not in the fp8 forward's rounding."""
    from bpe_transformer.ops import gemm

    gemm._AUTOTUNE = False
    gemm._route.clear()
    ids, vocab = P._tokens()
    model = P._ours(vocab, c, dev)
    model.enable_fp8()
    eng = P._engine(model, 1, c)
    data = P._batches(ids, P.STEPS, c.B, c.S, dev)
    out = {}
    for it in range(max(steps) + 1):
        if it in steps:
            with torch.no_grad():
                x, y = data[it]
                saved = [layer.fp8 for layer in model.layers]
                for layer in model.layers:
                    layer.fp8 = None
                lb = float(model.loss(x, y))
                for layer, f in zip(model.layers, saved):
                    layer.fp8 = f
            out[it] = {"bf16_eval_of_fp8_weights": lb}
            print(json.dumps({"cross_step": it, "bf16_eval_of_fp8_weights": round(lb, 4)}), flush=True)
        loss = eng.train_step([data[it]], lr=P._lr(it, c))
        if it in steps:
            out[it]["fp8_train_loss"] = float(loss)
            print(json.dumps({"cross_step": it, "fp8_train_loss": round(float(loss), 4)}), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--margins", default="1,2")
    ap.add_argument("--history", type=int, default=16)
    ap.add_argument("--bf16-wgrad", action="store_true")
    ap.add_argument("--out", default="gpurun_out/fp8_spike_probe.json")
    ap.add_argument("--same-weights", default="", help="steps (comma list): the same-weights evaluation only")
    ap.add_argument("--cross", default="", help="steps (comma list): bf16 evaluation of the fp8-trained weights")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = P.SHAPES["llama"]
    if a.cross:
        res = cross(c, [int(x) for x in a.cross.split(",")], dev)
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f)
        return
    if a.same_weights:
        res = same_weights(c, [int(x) for x in a.same_weights.split(",")], dev)
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f)
        return
    base, _ = run(c, False, 1.0, a.history, True, dev)
    out = {"steps": P.STEPS, "bf16": base, "runs": {}}
    for m in [float(x) for x in a.margins.split(",")]:
        l8, traces = run(c, True, m, a.history, not a.bf16_wgrad, dev)
        rel = [(x - y) / y for x, y in zip(l8, base)]
        worst = sorted(range(len(rel)), key=lambda i: -abs(rel[i]))[:6]
        sat = {}
        for i in worst:
            hits = []
            for tr in traces:
                n = len(tr["names"])
                for s, r in enumerate(tr["ratio"][i]):
                    if r > 1.0:
                        hits.append(f"L{s // n}.{tr['names'][s % n]}:{r:.2f}")
            sat[i] = hits
        nsat = [sum(1 for tr in traces for r in tr["ratio"][i] if r > 1.0) for i in range(len(l8))]
        key = f"margin{m:g}"
        out["runs"][key] = {"fp8": l8, "rel": rel, "max_rel": max(abs(x) for x in rel), "final_rel": rel[-1],
                            "saturated_slots_per_step": nsat, "worst_steps": {str(k): v for k, v in sat.items()},
                            "traces": traces}
        print(json.dumps({"run": key, "max_rel": round(max(abs(x) for x in rel), 4), "final_rel": round(rel[-1], 5),
                          "steps_with_saturation": sum(1 for x in nsat if x),
                          "worst": {k: (round(rel[k], 4), v) for k, v in sat.items()}}), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
