"""Back-to-back single-layer LSTM forwards through the C ABI (avc_lstm_forward), each output
cloned on the stream, compared with the first call after one host sync.  Shapes: decoder lstm1
(T=128, B=64, din=320, H=512) and one H=1024 layer; a 512x512 conv GEMM between calls (argv[1] ==
"conv") mimics the forward's neighbours."""
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: E402

from autovc_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(5)
with_conv = len(sys.argv) > 1 and sys.argv[1] == "conv"
for (T, B, din, H) in [(128, 64, 320, 512), (128, 64, 512, 1024), (128, 256, 320, 512)]:
    x = (torch.rand(T * B, din, generator=g) - 0.5).to(dev)
    s = 1.0 / H ** 0.5
    w = [((torch.rand(*shape, generator=g) * 2 - 1) * s).to(dev)
         for shape in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
    W = ((torch.rand(512, 512, 5, generator=g) - 0.5) * 0.1).to(dev)
    a = torch.rand(T * B, 512, generator=g).to(dev)
    bz, on = torch.zeros(512, device=dev), torch.ones(512, device=dev)
    outs = []
    with torch.no_grad():
        for i in range(30):
            y = torch.empty(T * B, H, device=dev)
            ops._lstm_fwd(x, *w, y, 0, H, False, False, T, B)
            outs.append(y.clone())
            if with_conv:
                ops.ConvBNAct.apply(a, W, bz, on, bz, None, None, True, 0.1, 1e-5, 1, None, T, B)
            if i == 0:
                torch.cuda.synchronize()
    torch.cuda.synchronize()
    d = [(o - outs[0]).abs().max().item() for o in outs]
    print(f"T={T} B={B} din={din} H={H} conv={with_conv}: calls differing from call 0: "
          f"{sum(v != 0 for v in d)} of 29; max {max(d):.2e}", flush=True)
