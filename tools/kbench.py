"""Kernel micro-benchmarks at the bench workload's shapes (large-proxy, cbox N=5633, 512^2).

python tools/kbench.py [attn|gemm|conv|all]   — prints achieved TFLOP/s per kernel (HIP events, 20 reps)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from renderformer_amd import ops  # noqa: E402
from renderformer_amd._lib import load  # noqa: E402

load()
dev = "cuda"
S, R, D, H, F = 5649, 4096, 1024, 8, 4096


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def attn_check():
    """numerics of the selected attention kernel vs torch fp32 (two problems, ragged tails)"""
    g = torch.Generator(device=dev).manual_seed(0)
    lens = [1000, 333]
    T = sum(lens)
    qkv = torch.randn(T, 3 * D, device=dev, generator=g).bfloat16()
    out = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    prob = torch.tensor([[0, 1000, 0, 1000, 0], [1000, 333, 1000, 333, 1000]], dtype=torch.int32, device=dev)
    worst = 0.0
    for sp in (0, 1, 3):
        ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], out, prob, 1000, H, n_split=sp)
        st = 0
        for n in lens:
            q, k, v = (qkv[st:st + n, i * D:(i + 1) * D].float().view(n, H, 128).transpose(0, 1) for i in range(3))
            ref = torch.softmax(q @ k.transpose(1, 2) / math.sqrt(128), -1) @ v
            got = out[st:st + n].float().view(n, H, 128).transpose(0, 1)
            worst = max(worst, float((got - ref).norm() / ref.norm()))
            st += n
    print(f"attn check rel-L2 worst {worst:.2e} ({'OK' if worst < 1e-2 else 'FAIL'})")


def attn():
    """stream-K kernel (n_split 0, q pre-scaled as in the model) vs the legacy per-unit kernel with splits."""
    attn_check()
    qkv = (torch.randn(S, 3 * D, device=dev) * 2).bfloat16()
    qs = (qkv[:, :D].float() * ops.Q_LOG2_SCALE).bfloat16()
    out = torch.empty(S, D, device=dev, dtype=torch.bfloat16)
    prob = torch.tensor([[0, S, 0, S, 0]], dtype=torch.int32, device=dev)
    fl = 4 * S * S * D
    ms = timeit(lambda: ops.attention(qs, qkv[:, D:2 * D], qkv[:, 2 * D:], out, prob, S, H, q_prescaled=True))
    print(f"attn stage1 S={S} stream-K (prescaled q): {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF")
    ms = timeit(lambda: ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], out, prob, S, H, n_split=0))
    print(f"attn stage1 S={S} stream-K (scale mult): {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF")
    for sp in (1, 4):
        ms = timeit(lambda: ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], out, prob, S, H, n_split=sp))
        print(f"attn stage1 S={S} legacy split={sp}: {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF")
    q = torch.randn(R, D, device=dev).bfloat16()
    q2 = (q.float() * ops.Q_LOG2_SCALE).bfloat16()
    kv = torch.randn(S, 2 * D, device=dev).bfloat16()
    prob2 = torch.tensor([[0, R, 0, S, 0]], dtype=torch.int32, device=dev)
    o2 = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
    fl = 4 * R * S * D
    ms = timeit(lambda: ops.attention(q2, kv[:, :D], kv[:, D:], o2, prob2, R, H, q_prescaled=True))
    print(f"attn cross R={R} S={S} stream-K: {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF")
    for sp in (1, 2):
        ms = timeit(lambda: ops.attention(q, kv[:, :D], kv[:, D:], o2, prob2, R, H, n_split=sp))
        print(f"attn cross R={R} S={S} legacy split={sp}: {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF")
    qkv2 = torch.randn(R, 3 * D, device=dev).bfloat16()
    for sh in (0, 4):
        ms = timeit(lambda: ops.swin_attention(qkv2[:, :D], qkv2[:, D:2 * D], qkv2[:, 2 * D:], o2, 1, 64, 64, sh, H))
        print(f"swin shift={sh}: {ms*1e3:8.1f} us  {4*R*64*D/ms/1e9:7.1f} TF")


def check(a, w, epi):
    """relative error of one fresh call vs an fp32 torch reference (SwiGLU: interleaved 16-row groups)"""
    m, n = a.shape[0], w.shape[0]
    ref = a.float() @ w.float().t()
    if epi == ops.EPI_SWIGLU:
        g = ref.view(m, n // 32, 2, 16)
        ref = (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(m, n // 2)
        c = torch.empty(m, n // 2, device=dev, dtype=torch.bfloat16)
    elif epi == ops.EPI_BF16:
        c = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    else:
        c0 = torch.randn(m, n, device=dev)
        c = c0.clone()
        if epi == ops.EPI_ADD_F32:
            ref = ref + c0
    ops.gemm(a, w, c, None, epi)
    return float((c.float() - ref).norm() / ref.norm())


def gemm():
    shapes = [("s1 qkv", S, 3 * D, D, ops.EPI_BF16), ("s1 out", S, D, D, ops.EPI_ADD_F32),
              ("s1 w13", S, 2 * F, D, ops.EPI_SWIGLU), ("s1 w2", S, D, F, ops.EPI_ADD_F32),
              ("s2 q", R, D, D, ops.EPI_BF16), ("s2 kv", S, 2 * D, D, ops.EPI_BF16),
              ("s2 w13", R, 2 * F, D, ops.EPI_SWIGLU), ("s2 w2", R, D, F, ops.EPI_ADD_F32),
              ("tex", 5633, D, 13312, ops.EPI_F32), ("sq8k", 8192, 8192, 8192, ops.EPI_BF16),
              ("s1 w13bf", S, 2 * F, D, ops.EPI_BF16), ("s2 w13bf", R, 2 * F, D, ops.EPI_BF16),
              ("s2 qkv", R, 3 * D, D, ops.EPI_BF16), ("s2 out", R, D, D, ops.EPI_ADD_F32),
              ("kvall", S, 20 * D, D, ops.EPI_BF16), ("ray", R, D, 192, ops.EPI_F32), ("vn", 5633, D, 128, ops.EPI_F32)]
    if os.environ.get("KB_SHAPES"):
        shapes = [x for x in shapes if x[0] in os.environ["KB_SHAPES"].split(",")]
    for name, m, n, k, epi in shapes:
        a = torch.randn(m, k, device=dev).bfloat16()
        w = (torch.randn(n, k, device=dev) / math.sqrt(k)).bfloat16()
        if epi == ops.EPI_SWIGLU:
            c = torch.empty(m, n // 2, device=dev, dtype=torch.bfloat16)
        elif epi == ops.EPI_BF16:
            c = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        else:
            c = torch.zeros(m, n, device=dev)
        variants = [("dp128", "128", None, "0"), ("dp128s4", "1284", None, "0"), ("dp128s5", "1285", None, "0"),
                    ("dp256x128", "2561", None, "0"), ("dp256ring", "256", None, "0"), ("dp256ph", "256", None, "0"),
                    ("dp128x256ph", "1282", None, "0"),
                    ("sk128x512", "128", "512", "0"), ("sk128x768", "128", "768", "0"), ("sk256", None, None, "1"),
                    ("skph", None, None, "0"), ("auto", None, None, None),
                    ("dp96x256", "962", None, "0"), ("dp64x256", "642", None, "0"), ("dp64x256w4", "644", None, "0"),
                    ("ph96x256", "963", None, "0"), ("ph64x256", "643", None, "0")]
        if os.environ.get("KB_VARIANTS"):
            variants = [v for v in variants if v[0] in os.environ["KB_VARIANTS"].split(",")]
        for label, tile, sk, gm in variants:
            for key, val in (("RF_GEMM_TILE", tile), ("RF_GEMM_SK", sk), ("RF_GEMM_SK256", gm)):
                if val is None:
                    os.environ.pop(key, None)
                else:
                    os.environ[key] = val
            os.environ["RF_GEMM_PHASED"] = "0" if label in ("dp256ring", "sk256") else "1"
            if label == "skph":
                os.environ["RF_GEMM_SKPH"] = "1"
            elif label == "auto":
                os.environ.pop("RF_GEMM_SKPH", None)
            else:
                os.environ["RF_GEMM_SKPH"] = "0"
            if label in ("dp256ring", "dp256ph", "sk256", "skph", "dp128x256ph") and n % 256:
                continue
            ms = timeit(lambda: ops.gemm(a, w, c, None, epi), reps=10 if k > 8000 else 20)
            err = check(a, w, epi)
            print(f"gemm {name:8s} {m}x{n}x{k} {label}: {ms*1e3:8.1f} us  {2*m*n*k/ms/1e9:7.1f} TF  relerr {err:.1e}",
                  flush=True)
        wt = w.t()
        ms = timeit(lambda: torch.matmul(a, wt), reps=10 if k > 8000 else 20)
        print(f"gemm {name:8s} {m}x{n}x{k} torch.matmul reference (vendor library, bf16 out): {ms*1e3:8.1f} us  {2*m*n*k/ms/1e9:7.1f} TF")
    a = torch.randn(8192, 8192, device=dev).bfloat16()
    b = torch.randn(8192, 8192, device=dev).bfloat16()
    ms = timeit(lambda: a @ b, reps=10)
    print(f"torch.matmul 8192^3 reference: {2*8192**3/ms/1e9:7.1f} TF")


def norms():
    """Row kernels at the frame's shapes: RMSNorm (f32 -> bf16) and q/k norm + RoPE (bf16 in place)."""
    for rows in (S, R):
        x = torch.randn(rows, D, device=dev)
        w = torch.rand(D, device=dev)
        o = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: ops.rmsnorm(x, w, 1e-6, o), reps=50)
        print(f"rmsnorm {rows}x{D}: {ms*1e3:6.1f} us  {rows*D*6/ms/1e6:6.0f} GB/s", flush=True)
    freqs = torch.rand(6, device=dev)
    for name, rows, seg in (("s1 qk", S, 2), ("s2 q", R, 1)):
        qkv = torch.randn(rows, 3 * D, device=dev).bfloat16()
        pair = qkv[:, :seg * D]
        nw = torch.rand(seg * D, device=dev)
        pos = torch.randn(rows, 9, device=dev)
        # the q/k pair as two one-segment groups (default) vs one two-segment wave (RF_QKN_SPLIT=0), interleaved
        for rep in range(2):
            for split in (("1", "0") if seg == 2 else ("1",)):
                os.environ["RF_QKN_SPLIT"] = split
                ms = timeit(lambda: ops.qk_norm_rope(pair, pair, H, nw, 1e-6, pos, freqs, n_seg=seg), reps=50)
                print(f"qk_norm_rope {name} {rows}x{seg*D} split={split}: {ms*1e3:6.1f} us  "
                      f"{rows*seg*D*4/ms/1e6:6.0f} GB/s", flush=True)
        os.environ.pop("RF_QKN_SPLIT", None)


def conv():
    from renderformer_amd.dpt import _Conv, split_planes
    for f16 in (True,) if os.environ.get("KB_F16_ONLY") else (True, False):
        shapes = [(256, 256, 256), (256, 128, 512), (256, 256, 128), (256, 256, 64), (256, 256, 32),
                  (128, 256, 256), (128, 32, 512), (512, 256, 128), (1024, 256, 64), (1024, 256, 32)]
        if os.environ.get("KB_CONV_HW"):  # only these output resolutions
            shapes = [x for x in shapes if str(x[2]) in os.environ["KB_CONV_HW"].split(",")]
        for cin, cout, hw in shapes:
            ks = int(os.environ.get("KB_CONV_K", "3"))  # kernel size (1: the 1x1 out_conv / projections)
            conv = _Conv(torch.randn(cout, cin, ks, ks) / 48, torch.randn(cout), dev, f16=f16)
            x = split_planes(torch.randn(1, hw, hw, cin, device=dev), conv.cin_pad, f16=f16)
            fl = 2 * hw * hw * cin * cout * ks * ks
            mf = 1 if f16 else 3
            tiles = os.environ.get("KB_CONV_TILES", "128,1288,256,2561,auto4w,auto").split(",") if f16 else ("128", "256")
            for t in tiles:
                os.environ["RF_CONV_PHASED"] = "1" if t == "256ph" else "0"
                os.environ["RF_CONV_SKW8"] = "0" if t == "auto4w" else "1"
                # h2 / h2s3 / h2s5: the 16 x 32-pixel halo kernel (4- / 3- / 5-deep W ring); other labels run without it
                os.environ["RF_CONV_HALO2"] = "1" if t.startswith("h2") or t.startswith("h3") else "0"
                os.environ["RF_CONV_HALO3"] = "1" if t.startswith("h3") else "0"  # h3: halo3_kernel (W from L2)
                os.environ["RF_H3_DBG"] = t[4:] if t.startswith("h3db") else "0"  # h3db1/2/4/8: ablations
                os.environ["RF_CONV_H2S"] = t[4:] if t.startswith("h2s") else "4"
                os.environ["RF_H2_DBG"] = t[4:] if t.startswith("h2db") else "0"  # h2db1/2/3: ablations
                os.environ["RF_CONV_HK"] = "1" if t == "hk" else "0"  # hk: conv3x3_hk_kernel (4 waves, one barrier per chunk)
                if not t.startswith("auto") and not t.startswith("h2") and t != "hk" and not t.startswith("h3"):
                    os.environ["RF_CONV_TILE"] = t.replace("ph", "")
                ms = timeit(lambda: conv(x, out_f32=True), reps=10)
                os.environ.pop("RF_CONV_TILE", None)
                print(f"conv{ks}x{ks} {'f16 ' if f16 else 'bf16x3'} {cin}->{cout} @{hw} tile={t}: "
                      f"{ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF(algorithmic)  {mf*fl/ms/1e9:7.1f} TF(MFMA issued)")
            if f16 and os.environ.get("KB_CONV_GEMM"):  # the same M, N, K as a plain bf16 GEMM (no gather)
                a = torch.randn(hw * hw, 9 * cin, device=dev).bfloat16()
                w = torch.randn(cout, 9 * cin, device=dev).bfloat16()
                c = torch.empty(hw * hw, cout, device=dev)
                for be in ("hip", "auto"):
                    os.environ["RF_GEMM_BACKEND"] = be
                    ms = timeit(lambda: ops.gemm(a, w, c, None, ops.EPI_F32), reps=10)
                    print(f"  plain GEMM {hw*hw}x{cout}x{9*cin} [{be}]: {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF")
                os.environ.pop("RF_GEMM_BACKEND", None)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    for name, fn in (("attn", attn), ("gemm", gemm), ("conv", conv), ("norms", norms)):
        if what in (name, "all"):
            fn()


def skstamps():
    """Per-block timeline of the phased stream-K GEMM (RF_GEMM_STAMPS=1 build path): segment ends, publish /
    wait / epilogue ends in shader cycles from each block's start, for the shapes in KB_SHAPES (m,n,k,epi;...)."""
    import numpy as np
    os.environ["RF_GEMM_STAMPS"] = "1"
    os.environ["RF_GEMM_BACKEND"] = "hip"
    os.environ["RF_GEMM_SKPH"] = "1"
    spec = os.environ.get("KB_SK", "5649,1024,1024,2;5649,1024,4096,2;5649,3072,1024,0")
    for item in spec.split(";"):
        m, n, k, epi = (int(x) for x in item.split(","))
        a = torch.randn(m, k, device=dev).bfloat16()
        w = (torch.randn(n, k, device=dev) / math.sqrt(k)).bfloat16()
        c = torch.empty(m, n, device=dev, dtype=torch.bfloat16) if epi == 0 else torch.zeros(m, n, device=dev)
        ms = timeit(lambda: ops.gemm(a, w, c, None, epi), reps=20)
        torch.cuda.synchronize()
        ws = ops._gemm_workspace(a.device)
        off = (256 * 256 * 256 - 65536) * 4
        st = ws[off:off + 256 * 16 * 8].view(torch.int64).view(256, 16).cpu().numpy()
        t0 = st[:, 0].min()
        rel = np.where(st > 0, st - t0, 0)
        ends = rel.max(axis=1)
        print(f"skstamps {m}x{n}x{k} epi{epi}: {ms*1e3:.1f} us; block start spread {int(st[:,0].max()-t0)} cyc, "
              f"end median {int(np.median(ends))} max {int(ends.max())} cyc", flush=True)
        for b in list(range(0, 8)) + [int(np.argmax(ends))]:
            seq = [int(v) for v in rel[b] if v > 0 or v == 0]
            print(f"  block {b:3d}: " + " ".join(str(int(v)) for v in rel[b][:12] if v != 0 or True), flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "skstamps":
    skstamps()


def coldgemm():
    """The frame's projection GEMMs under frame-like cache state: operands rotate over enough copies
    (> 512 MB) that every call reads A and W from HBM (in the frame each layer's weights are read once per
    frame and A was written by the previous kernel).  KB_TILES: comma list of RF_GEMM_TILE codes (auto = the
    cost model's pick)."""
    shapes = [("s1 qkv", S, 3 * D, D, ops.EPI_BF16), ("s1 out", S, D, D, ops.EPI_ADD_F32),
              ("s1 w2", S, D, F, ops.EPI_ADD_F32), ("s2 q", R, D, D, ops.EPI_BF16),
              ("s2 qkv", R, 3 * D, D, ops.EPI_BF16), ("s2 out", R, D, D, ops.EPI_ADD_F32),
              ("s2 w2", R, D, F, ops.EPI_ADD_F32), ("kvall", S, 20 * D, D, ops.EPI_BF16),
              ("s1 w13", S, 2 * F, D, ops.EPI_SWIGLU), ("s2 w13", R, 2 * F, D, ops.EPI_SWIGLU)]
    if os.environ.get("KB_SHAPES"):
        shapes = [x for x in shapes if x[0] in os.environ["KB_SHAPES"].split(",")]
    tiles = os.environ.get("KB_TILES", "auto").split(",")
    # KB_GROUP_M: comma list of RF_GEMM_GROUP_M raster overrides tried for every tile code (- = the host's pick)
    groups = os.environ.get("KB_GROUP_M", "-").split(",")
    for name, m, n, k, epi in shapes:
        per = m * k * 2 + n * k * 2 + m * n * 4
        nrot = max(2, int((768 << 20) // per) + 1)
        sets = []
        for _ in range(nrot):
            a = torch.randn(m, k, device=dev).bfloat16()
            w = (torch.randn(n, k, device=dev) / math.sqrt(k)).bfloat16()
            c = (torch.empty(m, n, device=dev, dtype=torch.bfloat16) if epi == ops.EPI_BF16
                 else torch.empty(m, n // 2, device=dev, dtype=torch.bfloat16) if epi == ops.EPI_SWIGLU
                 else torch.zeros(m, n, device=dev))
            sets.append((a, w, c))
        for t in tiles:
            if t == "auto":
                os.environ.pop("RF_GEMM_TILE", None)
            else:
                os.environ["RF_GEMM_TILE"] = t
            for gm in groups:
                if gm == "-":
                    os.environ.pop("RF_GEMM_GROUP_M", None)
                else:
                    os.environ["RF_GEMM_GROUP_M"] = gm
                i = [0]

                def run():
                    a, w, c = sets[i[0] % nrot]
                    i[0] += 1
                    ops.gemm(a, w, c, None, epi)
                ms = timeit(run, reps=3 * nrot)
                err = check(sets[0][0], sets[0][1], epi)
                print(f"cold gemm {name:7s} {m}x{n}x{k} tile={t:5s} group_m={gm:>3s}: {ms*1e3:8.1f} us  "
                      f"{2*m*n*k/ms/1e9:7.1f} TF  relerr {err:.1e}  ({nrot} rotating operand sets)", flush=True)
        os.environ.pop("RF_GEMM_TILE", None)
        os.environ.pop("RF_GEMM_GROUP_M", None)
        del sets
        torch.cuda.empty_cache()


def mx8():
    """The MX fp8 GEMM (rf_gemm_mx8) against the engine on fp16 operands at config 5's stage-2 shapes (24 views at
    1024^2 have 393,216 ray rows; KB_MX8_ROWS rows here, default 98,304 = 6 views), operands resident (the fp8 study:
    what bounds rf_gemm_mx8).  KB_MX8_ONLY=1 runs only the fp8 legs (for counter passes)."""
    m = int(os.environ.get("KB_MX8_ROWS", "98304"))
    only = os.environ.get("KB_MX8_ONLY") == "1"
    for name, n, k, epi in (("s2 w2", D, F, ops.EPI_ADD_F32), ("s2 q", D, D, ops.EPI_BF16),
                            ("s2 w13", 2 * F, D, ops.EPI_SWIGLU)):
        a = torch.randn(m, k, device=dev).bfloat16()
        w = (torch.randn(n, k, device=dev) / math.sqrt(k)).bfloat16()
        ncol = n // 2 if epi == ops.EPI_SWIGLU else n
        odt = torch.float32 if epi == ops.EPI_ADD_F32 else torch.bfloat16
        c8 = torch.zeros(m, ncol, device=dev, dtype=odt)
        aq, wq = ops.quant_mx8(a), ops.MX8(*ops.mx8_quant_ref(w))
        fl = 2 * m * n * k
        ms = timeit(lambda: ops.gemm_mx8(aq, wq, c8, None, epi), reps=10)
        print(f"mx8  {name:7s} {m}x{n}x{k}: {ms*1e3:9.1f} us  {fl/ms/1e9:7.1f} TF  ({fl/ms/1e9/5000:.3f} of 5 PF fp8)",
              flush=True)
        if not only:
            msq = timeit(lambda: ops.quant_mx8(a, aq), reps=10)
            print(f"quant {name:7s} {m}x{k}: {msq*1e3:9.1f} us", flush=True)
            ah, wh = a.half(), w.half()
            ch = torch.zeros(m, ncol, device=dev, dtype=torch.float32 if epi == ops.EPI_ADD_F32 else torch.float16)
            msh = timeit(lambda: ops.gemm(ah, wh, ch, None, epi), reps=10)
            print(f"f16  {name:7s} {m}x{n}x{k}: {msh*1e3:9.1f} us  {fl/msh/1e9:7.1f} TF  ({fl/msh/1e9/2500:.3f} of 2.5 PF)",
                  flush=True)
        del a, w, c8, aq, wq
        torch.cuda.empty_cache()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "mx8":
    mx8()

if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "coldgemm":
    coldgemm()


def vendor():
    """STUDY ONLY (never linked into librfhip): the vendor GEMM library (torch.nn.functional.linear on fp16, i.e.
    hipBLASLt / rocBLAS) against the engine on the frame's projection shapes with fp16 operands and cold rotating
    operand sets (as coldgemm).  Run it under rocprofv3 --kernel-trace --stats to get the library's kernel names
    (tile shape, stream-K or not) and durations, and under --pmc FETCH_SIZE / TCC_HIT_sum,TCC_MISS_sum passes for its
    traffic.  The engine rows use 16-bit outputs (RF_EPI_F16) so both write the same bytes."""
    shapes = [("s1 qkv", S, 3 * D, D), ("s1 out", S, D, D), ("s1 w2", S, D, F), ("s1 w13", S, 2 * F, D),
              ("s2 q", R, D, D), ("s2 w2", R, D, F), ("s2 w13", R, 2 * F, D), ("s2 qkv", R, 3 * D, D),
              ("kvall", S, 20 * D, D), ("sq8k", 8192, 8192, 8192)]
    if os.environ.get("KB_SHAPES"):
        shapes = [x for x in shapes if x[0] in os.environ["KB_SHAPES"].split(",")]
    for name, m, n, k in shapes:
        per = m * k * 2 + n * k * 2 + m * n * 2
        nrot = max(2, int((768 << 20) // per) + 1)
        sets = [(torch.randn(m, k, device=dev).half(), (torch.randn(n, k, device=dev) / math.sqrt(k)).half(),
                 torch.empty(m, n, device=dev, dtype=torch.float16)) for _ in range(nrot)]
        i = [0]

        def eng():
            a, w, c = sets[i[0] % nrot]
            i[0] += 1
            ops.gemm(a, w, c)

        def lib():
            a, w, c = sets[i[0] % nrot]
            i[0] += 1
            torch.nn.functional.linear(a, w)  # fp16 [m, n] out (torch's caching allocator: no malloc per call)
        fl = 2 * m * n * k
        for label, fn in (("engine", eng), ("vendor", lib)):
            ms = timeit(fn, reps=3 * nrot)
            print(f"vendor-study {name:7s} {m}x{n}x{k} {label}: {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF "
                  f"({nrot} rotating operand sets, fp16 in, fp16 out)", flush=True)
        del sets
        torch.cuda.empty_cache()


def prenorm():
    """Deferred RMSNorm A/B (rf.h rf_gemm_add_prenorm / rf_gemm_rownorm) on the frame's shapes, fp16 operands, cold
    rotating operand sets: producer = residual GEMM + rf_rmsnorm (the row-kernel pair) vs the residual GEMM that also
    writes x * g and the row sums (and the residual GEMM alone); consumer = the projection from rf_rmsnorm's output
    vs the projection with the 1 / rms row scale in its epilogue.  Two interleaved rounds."""
    from renderformer_amd.model import _interleave_swiglu
    prod = [("s1 out", S, D, D), ("s1 w2", S, D, F), ("s2 out", R, D, D), ("s2 w2", R, D, F)]
    cons = [("s1 qkv", S, 3 * D, D, 0), ("s1 w13", S, 2 * F, D, 1), ("s2 q", R, D, D, 0), ("s2 qkv", R, 3 * D, D, 0),
            ("s2 w13", R, 2 * F, D, 1)]
    sel = os.environ.get("KB_SHAPES")
    eps = 1e-6
    for rnd in range(1):
        for name, m, n, k in prod:
            if sel and name not in sel.split(","):
                continue
            per = m * k * 2 + n * k * 2 + m * n * 6
            nrot = max(2, int((768 << 20) // per) + 1)
            sets = [(torch.randn(m, k, device=dev).half(), (torch.randn(n, k, device=dev) / math.sqrt(k)).half(),
                     torch.randn(m, n, device=dev), torch.empty(m, n, device=dev, dtype=torch.float16),
                     torch.empty(m, ops.PRENORM_SLOTS, device=dev)) for _ in range(nrot)]
            g = torch.rand(n, device=dev) + 0.5
            i = [0]

            def nxt():
                i[0] += 1
                return sets[i[0] % nrot]

            def plain():
                a, w, x, h, ss = nxt()
                ops.gemm(a, w, x, None, ops.EPI_ADD_F32)

            def pair():
                a, w, x, h, ss = nxt()
                ops.gemm(a, w, x, None, ops.EPI_ADD_F32)
                ops.rmsnorm(x, g, eps, h)

            def fused():
                a, w, x, h, ss = nxt()
                ops.gemm_add_prenorm(a, w, x, g, h, ss)
            plain_only = os.environ.get("KB_PLAIN_ONLY") == "1"  # (a library without the deferred-norm entry points)
            fns = [("gemm ADD alone", plain), ("gemm ADD + rmsnorm", pair)] + ([] if plain_only else
                                                                              [("gemm_add_prenorm", fused)])
            best = {lab: 1e9 for lab, _ in fns}
            for rep in range(4):
                for lab, fn in (fns if rep % 2 == 0 else fns[::-1]):
                    best[lab] = min(best[lab], timeit(fn, reps=2 * nrot))
            for lab, _ in fns:
                print(f"prenorm r{rnd} producer {name:7s} {m}x{n}x{k} {lab:20s}: {best[lab]*1e3:8.1f} us ({nrot} sets, "
                      f"best of 4 interleaved)", flush=True)
            del sets
            torch.cuda.empty_cache()
        for name, m, n, k, sw in cons:
            if sel and name not in sel.split(","):
                continue
            per = m * k * 2 + n * k * 2 + m * n * 2
            nrot = max(2, int((768 << 20) // per) + 1)
            odt = torch.float16 if sw else torch.bfloat16
            ncol = n // 2 if sw else n
            epi = ops.EPI_SWIGLU if sw else ops.EPI_BF16

            def mkw():
                w = (torch.randn(n, k, device=dev) / math.sqrt(k)).half()
                return _interleave_swiglu(w[: n // 2], w[n // 2:]) if sw else w
            sets = [(torch.randn(m, k, device=dev).half(), mkw(), torch.empty(m, ncol, device=dev, dtype=odt),
                     torch.rand(m, ops.PRENORM_SLOTS, device=dev) + 1.0) for _ in range(nrot)]
            i = [0]

            def nxt():
                i[0] += 1
                return sets[i[0] % nrot]

            def plain():
                h, w, o, ss = nxt()
                ops.gemm(h, w, o, None, epi)

            def rown():
                h, w, o, ss = nxt()
                ops.gemm_rownorm(h, w, o, ss, eps, epi)
            # interleaved A/B/A/B..., best of 4 each: the W13 shapes run at the chip's power limit, so whichever
            # variant is timed second in a block runs at a lower clock
            fns = [("gemm", plain)] + ([] if os.environ.get("KB_PLAIN_ONLY") == "1" else [("gemm_rownorm", rown)])
            best = {lab: 1e9 for lab, _ in fns}
            for rep in range(4):
                for lab, fn in (fns if rep % 2 == 0 else fns[::-1]):
                    best[lab] = min(best[lab], timeit(fn, reps=2 * nrot))
            for lab, _ in fns:
                print(f"prenorm r{rnd} consumer {name:7s} {m}x{n}x{k} {lab:20s}: {best[lab]*1e3:8.1f} us ({nrot} sets, "
                      f"best of 4 interleaved)", flush=True)
            del sets
            torch.cuda.empty_cache()


def quad():
    """The 4-wave 256x256 engine (RF_GEMM_QUAD=1 whole tiles / persistent, 2 stream-K) against the default pick on
    the 256-divisible frame shapes, fp16 operands, cold rotating operand sets; the SwiGLU shapes with the SwiGLU
    epilogue (as in the frame), the others with fp16 outputs."""
    from renderformer_amd.model import _interleave_swiglu
    shapes = [("s1 qkv", S, 3 * D, D, 0), ("s1 w13", S, 2 * F, D, 1), ("s2 w13", R, 2 * F, D, 1),
              ("s2 qkv", R, 3 * D, D, 0), ("kvall", S, 20 * D, D, 0), ("sq8k", 8192, 8192, 8192, 0),
              ("s1 w2", S, D, F, 0), ("s2 w2", R, D, F, 0), ("s1 out", S, D, D, 0), ("s2 out", R, D, D, 0)]
    if os.environ.get("KB_SHAPES"):
        shapes = [x for x in shapes if x[0] in os.environ["KB_SHAPES"].split(",")]
    # labels: "0" default pick, "1" / "2" quad whole tiles / stream-K with register staging, "1d" / "2d" the same with
    # LDS-DMA staging; "1@128x192" etc. picks the block tile (RF_GEMM_QUAD_TILE)
    modes = os.environ.get("KB_QUAD", "0,1,2,1d").split(",")
    for name, m, n, k, sw in shapes:
        per = m * k * 2 + n * k * 2 + m * n * 2
        nrot = max(2, int((768 << 20) // per) + 1)
        sets = []
        for _ in range(nrot):
            w = (torch.randn(n, k, device=dev) / math.sqrt(k)).half()
            if sw:
                w = _interleave_swiglu(w[: n // 2].cpu(), w[n // 2:].cpu()).to(dev)
            sets.append((torch.randn(m, k, device=dev).half(), w,
                         torch.empty(m, n // 2 if sw else n, device=dev, dtype=torch.float16)))
        i = [0]

        def run():
            a, w, c = sets[i[0] % nrot]
            i[0] += 1
            ops.gemm(a, w, c, None, ops.EPI_SWIGLU if sw else ops.EPI_BF16)
        fl = 2 * m * n * k
        for md in modes:
            lab, _, tile = md.partition("@")
            os.environ["RF_GEMM_QUAD"] = lab.rstrip("d")
            os.environ["RF_GEMM_QUAD_STG"] = "0" if lab.endswith("d") else "1"
            if tile:
                os.environ["RF_GEMM_QUAD_TILE"] = tile
            else:
                os.environ.pop("RF_GEMM_QUAD_TILE", None)
            ms = timeit(run, reps=3 * nrot)
            print(f"quad-study {name:7s} {m}x{n}x{k} RF_GEMM_QUAD={md}: {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF "
                  f"({nrot} rotating operand sets{', SwiGLU' if sw else ''})", flush=True)
        for e in ("RF_GEMM_QUAD", "RF_GEMM_QUAD_STG", "RF_GEMM_QUAD_TILE"):
            os.environ.pop(e, None)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "vendor":
    vendor()
if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "quad":
    quad()
if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "prenorm":
    prenorm()


def c32():
    """output_conv2 at 512^2 (128 -> 32 filters, 3x3, fp16 planes) with its fused head (SiLU -> 1x1 to 3 -> ELU ->
    10^x - 1, NHWC as in the frame): conv3x3_c32_kernel (RF_CONV_C32=1, default) vs the engine path (0), interleaved."""
    from renderformer_amd.dpt import _Conv, split_planes, LOG_DECODE
    conv = _Conv(torch.randn(32, 128, 3, 3) / 48, torch.randn(32), dev, f16=True)
    x = split_planes(torch.randn(1, 512, 512, 128, device=dev), conv.cin_pad, f16=True)
    wf, bf = torch.randn(3, 32, device=dev) / 8, torch.zeros(3, device=dev)
    fl = 2 * 512 * 512 * 128 * 32 * 9
    for rep in range(2):
        for env in ("1", "0"):
            os.environ["RF_CONV_C32"] = env
            ms = timeit(lambda: conv(x, final=(wf, bf, 1.0), final_flags=LOG_DECODE), reps=20)
            print(f"output_conv2 512^2 128->32 + head RF_CONV_C32={env}: {ms*1e3:7.1f} us  {fl/ms/1e9:7.1f} TF",
                  flush=True)
    os.environ.pop("RF_CONV_C32", None)
    # per-chunk cost vs the input's channel count: cin = 32 makes each LDS-DMA instruction one contiguous 1-KiB run
    # (16 whole pixels), cin = 64 / 128 / 256 reads 64-B slices of 128 / 256 / 512-B pixels
    if os.environ.get("KB_C32_CIN"):
        for cin in (32, 64, 128, 256):
            cv = _Conv(torch.randn(32, cin, 3, 3) / 48, torch.randn(32), dev, f16=True)
            xc = split_planes(torch.randn(1, 512, 512, cin, device=dev), cv.cin_pad, f16=True)
            ms = timeit(lambda: cv(xc, final=(wf, bf, 1.0), final_flags=LOG_DECODE), reps=20)
            print(f"output_conv2-shape 512^2 {cin}->32 + head: {ms*1e3:7.1f} us  {ms*1e3/(cin//32):6.1f} us per "
                  f"32-channel chunk  {2*512*512*cin*32*9/ms/1e9:7.1f} TF", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "c32":
    c32()
