"""Per-stage error budget of the conversion forward against float64 (margin at B = 1).

For every stage of the decoder + postnet chain (and the encoder as one stage) this measures, on
the same seeded weights and input:
  local   -- the stage fed the float64 chain's input (rounded to fp32), its output vs the float64
             stage: the error the stage itself adds (GPU, and the fp32 reference = the oracle in fp32);
  -> post -- that local error carried to mel_post through the float64 downstream stages: what the
             stage's own rounding costs at the output the 1e-4 bar is stated on;
  chain   -- the full chain's error at the stage output (GPU per-layer path, fp32 reference).
Usage: python scripts/error_budget.py [seed B T [xseed]] (defaults 2 1 128: the worst B = 1 margin case of
profiles/r04_margin.json; xseed = the input mel's seed, default 1; tests/test_gpu_margin.py's small
cases use 5 + seed).  Prints a table; writes gpurun_out/error_budget_s{seed}_B{B}_T{T}.json."""
import json
import os
import sys

REPO = __file__.rsplit("/", 2)[0]
sys.path.insert(0, REPO)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from autovc_amd import ops  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.auto_encoder.encoder import conv_bn as gpu_conv_bn  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402
from oracle import autovc_oracle as orc  # noqa: E402

seed, B, T = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (2, 1, 128)
xseed = int(sys.argv[4]) if len(sys.argv) > 4 else 1
dev = torch.device("cuda:0")
torch.set_num_threads(min(16, os.cpu_count() or 1))
sd32 = torch_state_dict(seed)
sd64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd32.items()}
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(sd32)
ae.to(dev).train()
x_np, co_np, ct_np = synthetic_mel(xseed, B, T), synthetic_embedding(101, B), synthetic_embedding(201, B)


# frames [T*B][C] (time-major, the HIP layout) <-> (B, T, C) / (B, C, T)
def btc(f):
    return f.reshape(T, B, -1).transpose(0, 1)


def frames(x_btc):
    return x_btc.transpose(0, 1).reshape(T * B, -1)


def o_lstm(sd, prefix, l):
    def run(f):
        p = [sd[f"{prefix}.{n}_l{l}"] for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
        H = p[1].shape[1]
        h0 = f.new_zeros(1, B, H)
        out, _, _ = torch.lstm(btc(f), (h0, h0.clone()), p, True, 1, 0.0, False, False, True)
        return frames(out)
    return run


def o_conv(sd, prefix, act):
    def run(f, res=None):
        bufs = {k: v.clone() for k, v in sd.items() if prefix in k and ("running" in k or "num_batches" in k)}
        y = orc.conv_bn(btc(f).transpose(1, 2), sd, prefix, True, bufs).transpose(1, 2)
        y = frames(y)
        y = torch.relu(y) if act == "relu" else torch.tanh(y) if act == "tanh" else y
        return y + res if res is not None else y
    return run


def o_linear(sd):
    w, b = sd["decoder.linear_projection.linear_layer.weight"], sd["decoder.linear_projection.linear_layer.bias"]
    return lambda f: F.linear(f, w, b)


def g_lstm(mod, l):
    return lambda f: ops.LSTMLayer.apply(f.contiguous(), *mod.layer(l), T, B, False)


def g_conv(seq, act):
    a = {"relu": ops.ACT_RELU, "tanh": ops.ACT_TANH, None: ops.ACT_NONE}[act]
    return lambda f, res=None: gpu_conv_bn(seq, f.contiguous(), T, B, a, None if res is None else res.contiguous())


def g_linear(lin):
    return lambda f: ops.Linear.apply(f.contiguous(), lin.weight, lin.bias)


dec, post = ae.decoder, ae.postnet
STAGES = [("dec.lstm1", o_lstm(sd64, "decoder.lstm1", 0), o_lstm(sd32, "decoder.lstm1", 0), g_lstm(dec.lstm1, 0))]
for i in range(3):
    p = f"decoder.convolutions.{i}"
    STAGES.append((f"dec.conv{i}", o_conv(sd64, p, "relu"), o_conv(sd32, p, "relu"), g_conv(dec.convolutions[i], "relu")))
for l in range(2):
    STAGES.append((f"dec.lstm2.l{l}", o_lstm(sd64, "decoder.lstm2", l), o_lstm(sd32, "decoder.lstm2", l),
                   g_lstm(dec.lstm2, l)))
STAGES.append(("dec.linear", o_linear(sd64), o_linear(sd32), g_linear(dec.linear_projection.linear_layer)))
for i in range(5):
    p, act = f"postnet.convolutions.{i}", ("tanh" if i < 4 else None)
    STAGES.append((f"post.conv{i}", o_conv(sd64, p, act), o_conv(sd32, p, act), g_conv(post.convolutions[i], act)))
MEL = 6    # index of the stage whose output is mel (dec.linear; the residual of the last one)
LAST = len(STAGES) - 1


def chain(fns, f, k0, mel=None):
    """Stages k0.. of the chain from input f; returns every stage output (mel kept for the residual)."""
    outs = {}
    for k in range(k0, len(STAGES)):
        f = fns[k](f, mel) if k == LAST else fns[k](f)
        if k == MEL:
            mel = f
        outs[k] = f
    return outs


o64 = [s[1] for s in STAGES]
o32 = [s[2] for s in STAGES]
gpu = [s[3] for s in STAGES]

# the encoder stage: decoder input = upsampled codes ++ c_trg (pure data movement after the codes)
x, co, ct = (torch.from_numpy(a) for a in (x_np, co_np, ct_np))


def dec_in(codes_a, codes_b, c_trg):
    e = orc.upsample(codes_a, codes_b, T)
    return frames(torch.cat((e, c_trg.unsqueeze(-1).expand(-1, -1, T)), dim=1).transpose(1, 2))


with torch.no_grad():
    a64, b64 = orc.encoder(sd64, x.double(), co.double(), True, {})
    din64 = dec_in(a64, b64, ct.double())
    a32, b32 = orc.encoder(sd32, x, co, True, {})
    din32 = dec_in(a32, b32, ct)
    ga, gb = ae.encoder(x.to(dev), co.to(dev))
    dinG = dec_in([v.cpu() for v in ga], [v.cpu() for v in gb], ct)
    ref = chain(o64, din64, 0)           # float64 chain
    r32 = chain(o32, din32, 0)           # fp32 reference chain
    g = chain(gpu, dinG.to(dev), 0)      # GPU per-layer chain
    # the fused forward returns (B, 80, T) mels: to frames [T*B][80] like the chains
    fused = [v.cpu().double().permute(2, 0, 1).reshape(T * B, -1) for v in ae(x.to(dev), co.to(dev), ct.to(dev))[:2]]
    ae.check_health()


def mx(a, b):
    return float((a.double().cpu() - b.double().cpu()).abs().max())


post64 = ref[LAST]
rows = []
rows.append({"stage": "encoder (-> decoder input)", "local_gpu": mx(dinG, din64), "local_ref": mx(din32, din64),
             "post_gpu": mx(chain(o64, dinG.double(), 0)[LAST], post64),
             "post_ref": mx(chain(o64, din32.double(), 0)[LAST], post64),
             "chain_gpu": mx(dinG, din64), "chain_ref": mx(din32, din64), "max_abs": float(din64.abs().max())})
with torch.no_grad():
    for k, (name, f64, f32, fg) in enumerate(STAGES):
        inp = din64 if k == 0 else ref[k - 1]
        mel64 = ref[MEL]
        if k == LAST:
            yg = fg(inp.float().to(dev), mel64.float().to(dev)).cpu().double()
            y3 = f32(inp.float(), mel64.float()).double()
        else:
            yg = fg(inp.float().to(dev)).cpu().double()
            y3 = f32(inp.float()).double()
        ae.check_health()

        def carried(y):  # the stage's own error carried to mel_post in float64
            if k == LAST:
                return mx(y, post64)
            return mx(chain(o64, y, k + 1, mel64 if k > MEL else (y if k == MEL else None))[LAST], post64)
        rows.append({"stage": name, "local_gpu": mx(yg, ref[k]), "local_ref": mx(y3, ref[k]),
                     "post_gpu": carried(yg), "post_ref": carried(y3),
                     "chain_gpu": mx(g[k], ref[k]), "chain_ref": mx(r32[k], ref[k]), "max_abs": float(ref[k].abs().max())})

hdr = f"{'stage':28s} {'|y|max':>8s} {'local GPU':>10s} {'local ref':>10s} {'->post GPU':>11s} {'->post ref':>11s} {'chain GPU':>10s} {'chain ref':>10s}"
print(f"seed {seed}, B = {B}, T = {T}: distances from float64 (max |d|)")
print(hdr)
for r in rows:
    print(f"{r['stage']:28s} {r['max_abs']:8.3f} {r['local_gpu']:10.2e} {r['local_ref']:10.2e} {r['post_gpu']:11.2e} "
          f"{r['post_ref']:11.2e} {r['chain_gpu']:10.2e} {r['chain_ref']:10.2e}")
summ = {"gpu_fused_vs_f64_mel_post": mx(fused[1], post64), "gpu_per_layer_vs_f64_mel_post": mx(g[LAST], post64),
        "ref_vs_f64_mel_post": mx(r32[LAST], post64), "gpu_fused_vs_ref_mel_post": mx(fused[1], r32[LAST]),
        "gpu_fused_vs_per_layer_mel_post": mx(fused[1], g[LAST])}
print(json.dumps(summ, indent=1))
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
with open(os.path.join(REPO, "gpurun_out", f"error_budget_s{seed}_B{B}_T{T}_x{xseed}.json"), "w") as fh:
    json.dump({"seed": seed, "xseed": xseed, "B": B, "T": T, "rows": rows, "summary": summ}, fh, indent=1)
