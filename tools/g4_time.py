import os, sys, torch
sys.path.insert(0, os.getcwd())
import mmfd.kernels as K
dev = torch.device("cuda", 0)
for name, M, N, Kd in (("bert qkv", 65536, 2304, 768), ("bert out", 65536, 768, 768), ("bert ffn1", 65536, 3072, 768),
                       ("bert ffn2", 65536, 768, 3072), ("vit qkv", 100864, 2304, 768), ("vit ffn1", 100864, 3072, 768),
                       ("vit ffn2", 100864, 768, 3072)):
  for data in ("randn", "zeros"):
      A = torch.randn(M, Kd, device=dev).bfloat16(); B = torch.randn(N, Kd, device=dev).bfloat16()
      if data == "zeros":
          A.zero_(); B.zero_()
      bias = torch.randn(N, device=dev)
      res = {}
      for g4 in ("1", "0"):
          K.set_g4_mode("on" if g4 == "1" else "off")
          for _ in range(3): K.gemm(A, B, bias=bias)
          torch.cuda.synchronize()
          e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
          e0.record()
          for _ in range(20): out = K.gemm(A, B, bias=bias)
          e1.record(); torch.cuda.synchronize()
          res[g4] = (e0.elapsed_time(e1) / 20, out)
      for _ in range(3): torch.matmul(A, B.t())
      torch.cuda.synchronize()
      e0.record()
      for _ in range(20): torch.matmul(A, B.t())
      e1.record(); torch.cuda.synchronize()
      lib = e0.elapsed_time(e1) / 20
      same = torch.equal(res["1"][1], res["0"][1])
      fl = 2 * M * N * Kd
      print(f"{name:10s} {data:5s} M {M:6d} N {N:5d} K {Kd:5d}  g4 {res['1'][0]*1e3:7.1f} us ({fl/res['1'][0]/1e9:6.1f} TF)  "
            f"g8 {res['0'][0]*1e3:7.1f} us  hipBLASLt(no bias) {lib*1e3:7.1f} us  g4/g8 bitwise equal: {same}", flush=True)

# the step's epilogues: FFN1 (bias + GELU, pre-activation to aux), attention-out / FFN2 (bias +
# dropout + residual for BERT, bias + residual for ViT)
seed = K.Seed(1234) if hasattr(K, "Seed") else None
for name, M, N, Kd, mode in (("bert ffn1 gelu+aux", 65536, 3072, 768, "gelu"), ("bert out drop+res", 65536, 768, 768, "dropres"),
                             ("bert ffn2 drop+res", 65536, 768, 3072, "dropres"), ("vit ffn1 gelu+aux", 100864, 3072, 768, "gelu"),
                             ("vit ffn2 res", 100864, 768, 3072, "res")):
    A = torch.randn(M, Kd, device=dev).bfloat16(); B = torch.randn(N, Kd, device=dev).bfloat16()
    bias = torch.randn(N, device=dev)
    res_t = torch.randn(M, N, device=dev).bfloat16()
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    kw = dict(bias=bias)
    if mode == "gelu":
        kw.update(act=K.ACT_GELU, aux=aux)
    elif mode == "dropres":
        kw.update(residual=res_t, dropout_p=0.1, seed=seed, salt=7)
    else:
        kw.update(residual=res_t)
    res = {}
    for g4 in ("1", "0"):
        K.set_g4_mode(("gelu" if mode == "gelu" else "on") if g4 == "1" else "off")
        for _ in range(3): K.gemm(A, B, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20): out = K.gemm(A, B, **kw)
        e1.record(); torch.cuda.synchronize()
        res[g4] = (e0.elapsed_time(e1) / 20, out.clone(), aux.clone())
    same = torch.equal(res["1"][1], res["0"][1]) and (mode != "gelu" or torch.equal(res["1"][2], res["0"][2]))
    print(f"{name:20s} M {M:6d} N {N:5d} K {Kd:5d}  g4 {res['1'][0]*1e3:7.1f} us  g8 {res['0'][0]*1e3:7.1f} us  "
          f"bitwise equal: {same}", flush=True)
