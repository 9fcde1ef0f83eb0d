"""Benchmark: claim-evidence pairs/sec of the full fine-tune training step (BASELINE config 3:
bert-base-uncased + ViT-B/16 + fusion head, forward + backward + AdamW, bs=256 per GPU, 128 tokens,
224x224 images, synthetic data already resident in HBM), data parallel over N GPUs (one process per
GPU, RCCL gradient all-reduce). Prints ONE JSON line on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 256] [--precision fp32|bf16]
                  [--mode finetune|frozen] [--no-cpu-baseline] [--no-bf16]
                  [--workload train|forward|extract|retrieve|preprocess|latency|preembed|preembed_image]

The train headline is fp32 (the reference's arithmetic; logits within 1e-3 of the CPU oracle); the
same step in bf16 (bf16 MFMA operands, fp32 accumulation and master weights) is reported beside it
under "bf16". `--gpus N` outside a torch.distributed launcher starts N ranks itself.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# torch is imported in main(), not here: the corpus build's decode workers (mmfd.hostdecode, forkserver
# children) re-import this script as __mp_main__ and must stay torch-free
torch = dist = None

METRIC = "claim–evidence pairs/sec (fwd+bwd) at bs=256; 1/2/4/8 MI355X scaling"
GFLOP_PER_PAIR = {"finetune": 351.18, "frozen": 121.11}  # BASELINE.md §3 (FlopCounterMode, fwd+bwd)
PEAK_TFLOPS = {"bf16": 2516.6, "fp32": 157.3}  # MI355X dense MFMA (MI355X_MICROARCH.md)


def host_cores():
    """Threads for the CPU baseline: every core of the affinity mask, capped by the
    cgroup CPU quota when one is set (a GPU box grants a 16-CPU share of a larger machine; more
    threads than the quota only oversubscribe it)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def log(msg):
    """progress on stderr (the JSON line on stdout stays the only stdout output)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _timed(fn, steps):
    fn()  # warmup
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    return (time.perf_counter() - t0) / steps


def cpu_baseline(dev, steps=3, batch=4):
    """The oracle's CPU restatement (oracle/, validated against the reference's own fixtures) timed
    on this host with every core of the affinity mask: 1 warmup + `steps` timed steps
    of configs 1, 2 and 3 at bs=4. Config 2's oracle logits also give the measured full-size
    deviation of the HIP path's fp32 and bf16 logits (same weights and inputs)."""
    from oracle import encoders as OE
    from oracle import fusion_head as OF
    from oracle.fusion_head import init_params_like_reference
    from oracle.train_step import BERT_BASE, VIT_B16, OracleTrainer, bert_names, vit_names
    from mmfd.dataset import LABEL_TABLE, synthetic_batch
    from mmfd.model import MisinformationDetectionModel
    from mmfd.train import build_flagship

    cores = host_cores()
    torch.set_num_threads(cores)
    # training-mode dropout as the reference trains (p = 0.1 everywhere: model.py dropout=0.1 with
    # train.py:343-353, the HF encoders' hidden / attention dropout 0.1): torch's own dropout on the
    # oracle's sites, so the timed CPU step computes what the reference computes
    drop = lambda site, x: torch.nn.functional.dropout(x, 0.1, True)  # noqa: E731
    # config 3: full fine-tune step (the headline workload)
    head_names = [(k, list(v.shape)) for k, v in MisinformationDetectionModel(768, 768).state_dict().items()]
    tr = OracleTrainer(init_params_like_reference(bert_names(BERT_BASE), 1),
                       init_params_like_reference(vit_names(VIT_B16), 2),
                       init_params_like_reference(head_names, 3), drop=drop)
    b = synthetic_batch(batch, device="cpu", seed=7)
    log(f"cpu baseline: config 3 on {cores} threads")
    dt3 = _timed(lambda: tr.step(b), steps)
    del tr
    # config 2: dual encoder + head forward (eval), with the GPU deviation on the same inputs
    g2 = build_flagship(dev, "fp32", seed=3)
    sd = lambda m: {k: v.detach().float().cpu() for k, v in m.state_dict().items()}  # noqa: E731
    bp, vp, hp = sd(g2.text_encoder), sd(g2.image_encoder), sd(g2.head)
    b2 = synthetic_batch(batch, device="cpu", seed=17, ragged=True)

    def fwd2():
        with torch.no_grad():
            T = OE.bert_forward(bp, b2["input_ids"], b2["attention_mask"], None, num_layers=12, num_heads=12)
            I = OE.vit_forward(vp, b2["pixel_values"], num_layers=12, num_heads=12, patch=16)
            return OF.model_forward(hp, T[:batch], I[:batch], T[batch:], I[batch:], num_heads=8)

    log("cpu baseline: config 2")
    dt2 = _timed(fwd2, steps)
    want = torch.stack([y for pr in fwd2() for y in pr])
    dev_err = {}
    for prec in ("fp32", "bf16"):
        for m in (g2.text_encoder, g2.image_encoder, g2.head):
            m.set_precision(prec)
        got = g2.predict({k: v.to(dev) for k, v in b2.items()})
        got = torch.stack([y for pr in got for y in pr]).float().cpu()
        dev_err[prec] = float((got - want).abs().max())
    del g2
    # config 1: reference-default head training on pre-embedded inputs (train.py:343-356 dims)
    P1 = OF.xavier_like_reference([(k, list(v.shape)) for k, v in
                                   MisinformationDetectionModel(384, 1024).state_dict().items()], 5)
    P1 = {k: v.requires_grad_(True) for k, v in P1.items()}
    opt = torch.optim.AdamW(list(P1.values()), lr=1e-4)
    g = torch.Generator().manual_seed(9)
    Xt, Et = torch.randn(batch, 512, 384, generator=g), torch.randn(batch, 512, 384, generator=g)
    Xi, Ei = torch.randn(batch, 64, 1024, generator=g), torch.randn(batch, 64, 1024, generator=g)
    lab = LABEL_TABLE[torch.randint(0, 5, (batch,), generator=g)]

    def step1():
        opt.zero_grad(set_to_none=True)
        tot, _ = OF.path_loss(OF.model_forward(P1, Xt, Xi, Et, Ei, num_heads=8, drop=drop), lab)
        tot.backward()
        opt.step()

    log("cpu baseline: config 1")
    dt1 = _timed(step1, steps)
    out = {"value": round(batch / dt3, 4), "unit": "pairs/s", "cores": cores, "kind": "port",
           "sample": f"oracle/ CPU restatement (fp32 torch, {cores} threads = the affinity mask), bs={batch}, "
                     f"1 warmup + {steps} timed steps per config, training-mode dropout 0.1 (configs 1 and 3) as "
                     f"train.py trains; value = config 3 (full fine-tune step, {dt3:.2f} s/step)",
           "configs": {"config1_head_train_384_1024_L512_64": round(batch / dt1, 3),
                       "config2_forward_bert_vit_head": round(batch / dt2, 3),
                       "config3_finetune_step": round(batch / dt3, 4)}}
    parity = {"config2_fp32_max_abs_logit_err": dev_err["fp32"], "config2_bf16_max_abs_logit_err": dev_err["bf16"],
              "inputs": f"{batch} full-size pairs (ragged masks), same weights, eval"}
    return out, parity


# the PMC summaries taken on the current tree (tools/gpu_final.sh): looked up first, then the other
# committed summaries newest tag first (a kernel renamed since is then found under an older tag)
PMC_TAGS = ("r06zzzz_fp32", "r06zzzz_bf16")


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summaries (tools/profile.sh ->
    profiles/<tag>_hbm_traffic.json: FETCH_SIZE x2 + WRITE_SIZE): the current tree's (PMC_TAGS), else
    the newest that lists it, or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_traffic.json")))
    first = [os.path.join(ROOT, "profiles", f"{t}_hbm_traffic.json") for t in PMC_TAGS]
    files = [f for f in files if f not in first] + [f for f in reversed(first) if os.path.exists(f)]
    for path in reversed(files):
        with open(path) as f:
            k = json.load(f).get("kernels", {}).get(kernel)
        if k is not None:
            return int(k["traffic_bytes_per_dispatch"]), os.path.basename(path)
    return None, (os.path.basename(files[-1]) if files else None)


GFLOP_RESNET50, GFLOP_MPNET128 = 8.174, 22.35  # per image @224 / per sequence @L=128


def extract_leg(args, dev, world, rank, precision):
    """`--warmup` + `--steps` timed extractor steps of one precision on HBM-resident synthetic
    inputs (a step = `--batch` images through ResNet50 + `--batch` texts through MPNet at L=128),
    then the per-GEMM device times of one eager step (GemmProbe) for the roofline line."""
    from mmfd import kernels as K
    from mmfd.encoders import MPNetConfig, MPNetModel
    from mmfd.evidence import SentenceEncoder, resnet50

    torch.manual_seed(42)
    img = resnet50().to(dev).set_precision(precision)
    enc = SentenceEncoder(MPNetModel(MPNetConfig()), device=dev, precision=precision)
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    px = torch.randn(args.batch, 3, 224, 224, generator=g).to(dev)
    ids = torch.randint(3, 30527, (args.batch, 128), generator=g)
    ids[:, 0] = 0
    ids, mask = ids.to(dev), torch.ones_like(ids, device=dev)

    def step():
        f = img(px)
        e = enc.encode_ids(ids, mask, batch_size=args.batch)
        return f, e

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    t_img = t_txt = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e0.record()
        img(px)
        e1.record()
        enc.encode_ids(ids, mask, batch_size=args.batch)
        e2.record()
        e2.synchronize()
        t_img += e0.elapsed_time(e1)
        t_txt += e1.elapsed_time(e2)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    probe = K.GemmProbe()
    with probe:
        step()
    prof = probe.summary()
    dom_name, d = max(((k, v) for k, v in prof.items() if "split-K" not in k), key=lambda kv: kv[1]["ms"])
    achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
    x6 = "_x6f" in dom_name or dom_name.rstrip().endswith("true>")
    peak = PEAK_TFLOPS[precision] if not x6 else PEAK_TFLOPS["bf16"] / 6
    traffic, traffic_src = pmc_traffic(dom_name)
    ips = args.batch * args.steps / (t_img * 1e-3)
    tps = args.batch * args.steps / (t_txt * 1e-3)
    step_tf = args.batch * args.steps * (GFLOP_RESNET50 + GFLOP_MPNET128) / ((t_img + t_txt) * 1e-3) / 1e3
    del img, enc
    return {"items": 2 * args.batch * world * args.steps / elapsed, "ms": 1000.0 * elapsed / args.steps,
            "ips": ips, "tps": tps, "step_tflops": step_tf,
            "roofline": {"bound": "mfma", "kernel": dom_name, "achieved": round(achieved, 1), "peak": round(peak, 1),
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                         "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                         "launches_per_step": d["launches"], "avg_launch_us": round(1000.0 * d["ms"] / d["launches"], 2),
                         "algorithmic_flops_per_launch": int(d["flops"] // d["launches"]),
                         **({"peak_note": "split-operand fp32 ceiling: bf16 dense MFMA peak / 6"} if x6 else {})}}


def extract_cpu_baseline(n=4):
    """the oracle's ResNet50 (oracle/resnet.py) and MPNet (oracle/encoders.py) on `n` images @224 and
    `n` texts @L=128 on this host's cores (fp32, the reference's own arithmetic)"""
    from mmfd.encoders import MPNetConfig, MPNetModel
    from mmfd.evidence import resnet50
    from oracle import encoders as OE
    from oracle.resnet import resnet_forward
    cores = host_cores()
    torch.set_num_threads(cores)
    torch.manual_seed(42)
    P = {k: v.clone() for k, v in resnet50().state_dict().items()}
    M = {k: v.clone() for k, v in MPNetModel(MPNetConfig()).state_dict().items()}
    g = torch.Generator().manual_seed(5)
    x = torch.randn(n, 3, 224, 224, generator=g)
    ids = torch.randint(3, 30527, (n, 128), generator=g)
    ids[:, 0] = 0
    with torch.no_grad():
        ti = _timed(lambda: resnet_forward(P, x), 2)
        tt = _timed(lambda: OE.mpnet_forward(P=M, input_ids=ids, attention_mask=torch.ones_like(ids), num_layers=12,
                                             num_heads=12), 2)
    return {"value": round(2 * n / (ti + tt), 3), "unit": "items/s", "cores": cores, "kind": "port",
            "sample": f"oracle/ ResNet50 on {n} images @224 + MPNet on {n} texts @L=128 (fp32 torch, {cores} threads), "
                      f"1 warmup + 2 timed batches each",
            "images_per_s": round(n / ti, 3), "texts_per_s": round(n / tt, 3)}


def extract_e2e(dev, precision, n_img=2048, n_txt=4096):
    """config 5 end to end through the product API, from files: `ImageCorpus.create_feature_corpus`
    over `n_img` JPEG files (375x500, host decode on a process pool overlapping the GPU, the HIP
    "retrieval" preprocessing, ResNet50, the reference's pickle corpus written) and
    `TextCorpus.encode_corpus` over a `{split}_enriched.csv` of `n_txt` texts (a fast word-level
    tokenizer over a 30,527-entry vocabulary — the hub's MPNet vocabulary is not available offline —
    length-sorted batches, MPNet, the fp16 embedding store written). Synthetic files in a temp dir."""
    import tempfile

    import numpy as np
    import pandas as pd
    from PIL import Image
    from tokenizers import Tokenizer, models, pre_tokenizers, processors
    from transformers import PreTrainedTokenizerFast

    from mmfd.encoders import MPNetConfig, MPNetModel
    from mmfd.evidence import ImageCorpus, ImageSimilarity, SentenceEncoder, TextCorpus
    words = [f"w{i}" for i in range(30522)]
    vocab = {w: i for i, w in enumerate(["<s>", "<pad>", "</s>", "<unk>", "<mask>"] + words)}
    tk = Tokenizer(models.WordLevel(vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    tk.post_processor = processors.TemplateProcessing(single="<s> $A </s>", special_tokens=[("<s>", 0), ("</s>", 2)])
    tok = PreTrainedTokenizerFast(tokenizer_object=tk, pad_token="<pad>", unk_token="<unk>", bos_token="<s>",
                                  eos_token="</s>", mask_token="<mask>")
    rng = np.random.default_rng(3)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        os.makedirs(os.path.join(d, "imgs"))
        base = rng.integers(0, 256, (375, 500, 3), dtype=np.uint8)
        for i in range(n_img):
            Image.fromarray(np.roll(base, i * 7, axis=1)).save(os.path.join(d, "imgs", f"{i:05d}.jpg"), quality=90)
        texts = [" ".join(words[j] for j in rng.integers(0, 30522, int(rng.integers(20, 126)))) for _ in range(n_txt)]
        pd.DataFrame({"id": range(n_txt), "evidence_enriched": texts}).to_csv(os.path.join(d, "train_enriched.csv"),
                                                                             index=False)
        torch.manual_seed(42)
        corpus = ImageCorpus(os.path.join(d, "corpus.pkl"), extractor=ImageSimilarity(device=dev, precision=precision))
        tc = TextCorpus(d, "train", encoder=SentenceEncoder(MPNetModel(MPNetConfig()), device=dev, precision=precision,
                                                           tokenizer=tok, max_seq_length=128))
        warm = os.path.join(d, "warm")  # one small warm-up build (kernel attributes, allocator)
        os.makedirs(warm)
        for i in range(8):
            os.link(os.path.join(d, "imgs", f"{i:05d}.jpg"), os.path.join(warm, f"{i:05d}.jpg"))
        ImageCorpus(os.path.join(d, "w.pkl"), extractor=corpus.feature_extractor).create_feature_corpus(warm)
        tc.bi_encoder.encode(texts[:8])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        corpus.create_feature_corpus(os.path.join(d, "imgs"))
        t1 = time.perf_counter()
        tc.encode_corpus()
        t2 = time.perf_counter()
        assert len(corpus.feature_dict) == n_img
        # the round-3 thread-pool decode on the same files, and the host decode alone (the pool
        # without the GPU: the host-core bound of the image build)
        thr = ImageCorpus(os.path.join(d, "thr.pkl"), extractor=corpus.feature_extractor, decode="threads")
        t3 = time.perf_counter()
        thr.create_feature_corpus(os.path.join(d, "imgs"))
        t4 = time.perf_counter()
        assert all(torch.equal(thr.feature_dict[k], corpus.feature_dict[k]) for k in corpus.feature_dict)
        paths = sorted(os.path.join(d, "imgs", n) for n in os.listdir(os.path.join(d, "imgs")))
        ring = corpus._decode_ring()
        t5 = time.perf_counter()
        chunks = [paths[i:i + corpus.batch_size] for i in range(0, len(paths), corpus.batch_size)]
        h = ring.submit(chunks[0], 0)
        for ci in range(len(chunks)):  # the same decode + upload pipeline without the GPU's work
            ring.upload(h, ci % 2)
            if ci + 1 < len(chunks):
                h = ring.submit(chunks[ci + 1], (ci + 1) % 2)
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        workers = ring.workers
        corpus.close()
    cores = len(os.sched_getaffinity(0))
    return {"images_per_s": round(n_img / (t1 - t0), 1), "texts_per_s": round(n_txt / (t2 - t1), 1),
            "items_per_s": round((n_img + n_txt) / (t2 - t0), 1), "images": n_img, "texts": n_txt,
            "images_per_s_thread_decode": round(n_img / (t4 - t3), 1),
            "host_decode_upload_images_per_s": round(n_img / (t6 - t5), 1),
            "decode_workers": workers, "host_cores_visible": cores,
            "note": "ImageCorpus.create_feature_corpus over JPEG files (375x500 random-pixel q90: a heavy decode; "
                    "host decode on a forkserver process pool writing into a page-locked shared-memory ring, "
                    "asynchronous uploads, HIP preprocessing from the device copy; ResNet50; features kept on the "
                    "device until the end; pickle corpus written) + TextCorpus.encode_corpus over a "
                    "CSV (word-level fast tokenizer, length-sorted batches, MPNet, fp16 store written); "
                    "host_decode_upload = the same decode ring + uploads without the GPU's work (the host-core "
                    "bound: with 8 ranks per node each rank gets 1/8 of the node's cores for it)"}


def extract_main(args, dev, world, rank):
    """BASELINE config 5: evidence-corpus build — ResNet50 image features (im2im_retrieval.py:29-36)
    and MPNet CLS text embeddings at L=128 (text2text_retrieval.py:129-157), eval mode, random-init
    weights, fp32 (the reference's precision) with bf16 beside it; the headline times inputs
    resident in HBM (each rank its own shard, no collective), `e2e` the product API from files."""
    res = extract_leg(args, dev, world, rank, args.precision)
    log(f"extract {args.precision}: {res['items']:.1f} items/s")
    sec = None
    if args.precision == "fp32" and not args.no_bf16:
        torch.cuda.empty_cache()
        sec = extract_leg(args, dev, world, rank, "bf16")
        log(f"extract bf16: {sec['items']:.1f} items/s")
    e2e = None
    if world == 1 and not args.no_cpu_baseline:
        try:
            e2e = extract_e2e(dev, args.precision)
            log(f"extract e2e: {e2e}")
        except Exception as e:  # never hide the headline
            e2e = {"error": repr(e)}
    if rank == 0:
        out = {
            "metric": "evidence-corpus items/sec (ResNet50 image features + MPNet L=128 text embeddings)",
            "value": round(res["items"], 1), "unit": "items/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(res["ms"], 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic (random-init weights)",
            "config": {"workload": "evidence corpus build (BASELINE config 5): resnet50 @224 + multi-qa-mpnet-base "
                                   "@L=128, eval", "global_batch": args.batch * world, "parallelism": f"shard{world}"},
            "images_per_s_per_gpu": round(res["ips"], 1), "texts_per_s_per_gpu": round(res["tps"], 1),
            "image_tflops": round(res["ips"] * GFLOP_RESNET50 / 1e3, 1),
            "text_tflops": round(res["tps"] * GFLOP_MPNET128 / 1e3, 1),
            "roofline": res["roofline"],
            "roofline_step_frac": round(res["step_tflops"] / step_peak(args.precision)[0], 4),
            "roofline_step_peak": {"peak": round(step_peak(args.precision)[0], 1), "unit": "TFLOP/s",
                                   "note": step_peak(args.precision)[1] + f"; {GFLOP_RESNET50} GFLOP/image, "
                                           f"{GFLOP_MPNET128} GFLOP/text (SURVEY 8(d))"},
        }
        if sec is not None:
            out["bf16"] = {"value": round(sec["items"], 1), "unit": "items/s",
                           "images_per_s_per_gpu": round(sec["ips"], 1), "texts_per_s_per_gpu": round(sec["tps"], 1),
                           "roofline": sec["roofline"]}
        if e2e is not None:
            out["e2e"] = e2e
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = extract_cpu_baseline()
            except Exception as e:
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def retrieve_main(args, dev, world, rank):
    """evidence retrieval scoring — a batch of `--batch` query features against
    the reference's image corpus shape (41,256 ResNet50 features x 2048 fp32, resident in HBM;
    im2im_retrieval.py:80-106): cosine scores + exact top-50 candidates + the distinct-score
    filter. Each rank searches its own corpus shard (no collective). A step = one query batch."""
    from mmfd import kernels as K
    from mmfd.retrieval import CorpusIndex

    N, D, top_k = 41256, 2048, 50
    g = torch.Generator(device="cpu").manual_seed(77 + rank)
    feats = torch.randn(N, D, generator=g).abs_()
    index = CorpusIndex(feats, mode="pair", eps=1e-6, device=dev)
    q = torch.randn(args.batch, D, generator=g).abs_().to(dev)

    def step():
        return index.search(q, top_k)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    # dominant kernel: the score pass, timed with events on the launch stream (torch's current)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        sc = K.cosine_scores(q, index.emb, mode=K.COS_PAIR, eps=1e-6)
    e1.record()
    torch.cuda.synchronize()
    passes = (args.batch + 7) // 8  # one corpus pass per 8-query tile
    score_ms = e0.elapsed_time(e1) / reps
    algo_bytes = passes * N * D * 4 + args.batch * N * 4  # corpus read per pass + scores written
    e0.record()
    for _ in range(reps):
        K.topk(sc, 2 * top_k)
    e1.record()
    torch.cuda.synchronize()
    topk_ms = e0.elapsed_time(e1) / reps
    if rank == 0:
        qps = args.batch * world * args.steps / elapsed
        achieved = algo_bytes / (score_ms * 1e-3) / 1e9
        out = {
            "metric": "evidence retrieval queries/sec (cosine top-50, distinct scores)", "value": round(qps, 1),
            "unit": "queries/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (non-negative features)",
            "config": {"workload": "retrieval scoring (SURVEY 8f row 2): 41,256 x 2048 fp32 image corpus, top_k 50",
                       "global_batch": args.batch * world, "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "kernel": "cosine_scores_kernel<float>", "achieved": round(achieved, 1),
                         "peak": 8000.0, "unit": "GB/s", "frac": round(achieved / 8000.0, 4), "traffic": None,
                         "algorithmic_bytes_per_launch": algo_bytes, "avg_launch_us": round(1000 * score_ms, 2)},
            "topk_us": round(1000 * topk_ms, 2),
        }
        if not args.no_cpu_baseline and world == 1:
            from oracle.retrieval import cosine_pair, retrieve_unique
            fc, qc = feats.numpy(), q[:2].cpu().numpy()
            t1 = time.perf_counter()
            for i in range(len(qc)):
                retrieve_unique(cosine_pair(qc[i:i + 1], fc)[0], top_k)
            dt = (time.perf_counter() - t1) / len(qc)
            out["cpu_baseline"] = {"value": round(1.0 / dt, 2), "unit": "queries/s", "cores": torch.get_num_threads(),
                                   "kind": "port", "sample": "oracle/retrieval.py (numpy float64 scores, stable "
                                   "sort, distinct filter), 1-2 queries against the same 41,256 x 2048 corpus"}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def forward_main(args, dev, world, rank):
    """BASELINE config 2: bert-base-uncased + ViT-B/16 + fusion head forward only (eval), default
    bs=64 pairs per GPU, synthetic pairs resident in HBM; a step = one batch of pairs.
    Logit parity for this path: tests/test_trainer_gpu.py::test_config2_full_size_forward_logits."""
    from mmfd import kernels as K  # noqa: F401
    from mmfd.dataset import synthetic_batch
    from mmfd.train import build_flagship

    tr = build_flagship(dev, args.precision, seed=42 + rank)
    batch = synthetic_batch(args.batch, seed=1000 + rank, device=dev)
    for _ in range(args.warmup):
        tr.predict(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.predict(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    if rank == 0:
        pairs = args.batch * world * args.steps / elapsed
        tf = pairs / world * 117.21e9 / 1e12  # 117.21 GFLOP/pair forward
        out = {"metric": "claim-evidence pairs/sec (forward only, eval)", "value": round(pairs, 2), "unit": "pairs/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(1000.0 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": args.precision, "data": "synthetic (Factify-shaped pairs, random-init weights)",
               "config": {"workload": "config 2: bert-base-uncased + ViT-B/16 + fusion head forward (eval)",
                          "global_batch": args.batch * world, "seq_len": 128, "image_size": 224,
                          "parallelism": f"dp{world}"},
               "step_tflops_per_gpu": round(tf, 1), "roofline_step_frac": round(tf / step_peak(args.precision)[0], 4)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def preprocess_main(args, dev, world, rank):
    """raw-image preprocessing (dataset.py:14-19 transform: Resize(256) +
    CenterCrop(256) + ToTensor + Normalize) of `--batch` decoded 375x500 RGB images already in
    HBM -> the fp32 [B, 3, 256, 256] pixel tensor; bit-exact with PIL + torchvision
    (tests/test_preprocess_gpu.py). Each rank processes its own images (no collective)."""
    from mmfd.preprocess import ImagePreprocessor

    H, W = 375, 500
    pre = ImagePreprocessor("train", device=dev)
    g = torch.Generator(device="cpu").manual_seed(5 + rank)
    src = torch.randint(0, 256, (args.batch, H, W, 3), generator=g, dtype=torch.uint8).to(dev)
    plan = pre.plan([(H, W)] * args.batch, [src[i].data_ptr() for i in range(args.batch)])
    out = torch.empty(args.batch, 3, 256, 256, device=dev)
    for _ in range(args.warmup):
        pre.launch(plan, out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        pre.launch(plan, out)
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    if rank == 0:
        per = e0.elapsed_time(e1) / args.steps * 1e-3
        oh, ow = 256, 341
        # algorithmic bytes per image: source read, pass-1 rows written + read, fp32 output written
        algo = H * W * 3 + 2 * H * ow * 3 + 3 * 256 * 256 * 4
        achieved = algo * args.batch / per / 1e9
        out_d = {"metric": "images/sec preprocessed (Resize 256 + CenterCrop 256 + ToTensor + Normalize)",
                 "value": round(args.batch * world * args.steps / elapsed, 1), "unit": "images/s", "n_gpus": world,
                 "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
                 "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                 "data": "synthetic 375x500 RGB uint8 images resident in HBM",
                 "config": {"workload": "raw-image preprocessing (SURVEY 8f row 3), dataset.py:14-19 transform",
                            "global_batch": args.batch * world, "parallelism": f"shard{world}"},
                 "roofline": {"bound": "hbm", "kernel": "resize_h_kernel + resize_v_norm_kernel",
                              "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                              "frac": round(achieved / 8000.0, 4), "traffic": None,
                              "algorithmic_bytes_per_launch": algo * args.batch, "avg_launch_us": round(per * 1e6, 2)}}
        if not args.no_cpu_baseline and world == 1:
            from PIL import Image
            from oracle.preprocess import preprocess
            from mmfd.preprocess import MODES
            c = MODES["train"]
            imgs = [Image.fromarray(src[i].cpu().numpy()) for i in range(min(32, args.batch))]
            t1 = time.perf_counter()
            for im in imgs:
                preprocess(im, c["resize"], c["crop"], c["mean"], c["std"])
            dt = (time.perf_counter() - t1) / len(imgs)
            out_d["cpu_baseline"] = {"value": round(1.0 / dt, 1), "unit": "images/s", "cores": 1, "kind": "port",
                                     "sample": f"oracle/preprocess.py (PIL resize + numpy normalise), {len(imgs)} images, one thread"}
        print(json.dumps(out_d), flush=True)
    if world > 1:
        dist.destroy_process_group()


def latency_main(args, dev, world, rank):
    """single-pair inference of evaluate.py:95-192 (claim + evidence text padded
    to max_length 512, two 224x224 images, bert-base-uncased + ViT-B/16 + fusion head, eval) through
    mmfd.predict.PairPredictor (the engine under MisinformationPredictor); a step = one pair, inputs already resident in HBM. The
    HIP-graph replay is the value; the eager (per-kernel Python launch) latency is reported beside
    it. Each rank runs its own replica (no collective)."""
    from mmfd.predict import PairPredictor
    from mmfd.train import build_flagship

    tr = build_flagship(dev, args.precision, seed=42 + rank)
    g = torch.Generator(device="cpu").manual_seed(77 + rank)
    L = 512

    def pair():
        ids = torch.randint(1000, 30522, (L,), generator=g)
        ids[0], ids[-1] = 101, 102
        return ids.to(dev), torch.ones(L, dtype=torch.long, device=dev), torch.randn(3, 224, 224, generator=g).to(dev)

    c, e = pair(), pair()
    res = {}
    for mode in ("eager", "graph"):
        pr = PairPredictor.from_trainer(tr, use_graph=mode == "graph")
        for _ in range(max(1, args.warmup)):
            pr.predict_logits(*c, *e)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pr.predict_logits(*c, *e)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        res[mode] = t.item() / args.steps * 1e3
    if rank == 0:
        # algorithmic forward FLOPs of the pair at L=512 (FlopCounterMode-style matmul count):
        # BERT 2 x (12 x (4 x 512 x 768^2 x 2 + 2 x 512 x 768 x 3072 x 2 + 2 x 512^2 x 768 x 2)),
        # ViT 2 x 35.126 GFLOP, fusion head 2.266 GFLOP
        bert = 12 * (4 * 512 * 768 * 768 * 2 + 2 * 512 * 768 * 3072 * 2 + 2 * 512 * 512 * 768 * 2)
        flops = 2 * bert + 2 * 35.126e9 + 2.266e9
        out = {"metric": "single claim-evidence pair latency (evaluate.py path, L=512)",
               "value": round(res["graph"], 3), "unit": "ms/pair", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(res["graph"], 3), "higher_is_better": False,
               "scaling": "replicas", "vs_baseline": None, "dtype": args.precision,
               "data": "synthetic pair (512-token texts, 224x224 images, random-init weights)",
               "config": {"workload": "single-pair inference (SURVEY 8f row 4): bert-base-uncased + ViT-B/16 + "
                                      "fusion head, HIP graph replay", "global_batch": 1, "seq_len": L,
                          "image_size": 224, "parallelism": f"replicas{world}"},
               "eager_ms_per_pair": round(res["eager"], 3),
               "tflops_graph": round(flops / (res["graph"] * 1e-3) / 1e12, 1)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def preembed_main(args, dev, world, rank):
    """SURVEY §8(f) row 1, text side: the pre-embedding pass of preprocess_embeddings.py:63-80 —
    DeBERTa-v3-xsmall (the reference's text encoder) over texts padded to max_length 512, eval, no
    grad; a step = `--batch` sequences (default 64) resident in HBM. Each rank embeds its own shard
    of the corpus (no collective). Algorithmic work per sequence at L=512: 12 x (QKV 3LD^2 + out
    LD^2 + FFN 2LDI + attention 2L^2D + c2p/p2c 2L(2S)D) x 2 FLOP = 31.4 GFLOP (the per-batch
    projections of the 512 relative embeddings excluded)."""
    from mmfd.deberta import DebertaV2Config, DebertaV2Model

    L = 512
    B = args.batch
    torch.manual_seed(42 + rank)
    m = DebertaV2Model(DebertaV2Config()).to(dev).eval().set_precision(args.precision)
    g = torch.Generator(device="cpu").manual_seed(9 + rank)
    ids = torch.randint(1, 128100, (B, L), generator=g)
    n = torch.randint(32, L + 1, (B,), generator=g)
    mask = (torch.arange(L)[None] < n[:, None]).long()
    ids, mask = (ids * mask).to(dev), mask.to(dev)
    with torch.no_grad():
        for _ in range(args.warmup):
            m(input_ids=ids, attention_mask=mask)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            m(input_ids=ids, attention_mask=mask)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    if rank == 0:
        D, I, S = 384, 1536, 256
        flops = 12 * (3 * L * D * D + L * D * D + 2 * L * D * I + 2 * L * L * D + 2 * L * 2 * S * D) * 2
        seqs = B * world * args.steps / elapsed
        tf = seqs / world * flops / 1e12
        out = {"metric": "texts/sec embedded (DeBERTa-v3-xsmall, max_length 512, pre-embedding pass)",
               "value": round(seqs, 1), "unit": "sequences/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
               "data": "synthetic token ids (ragged 32..512 real tokens, padded to 512), random-init weights",
               "config": {"workload": "pre-embedding text pass (SURVEY 8f row 1): deberta-v3-xsmall forward",
                          "global_batch": B * world, "seq_len": L, "parallelism": f"shard{world}"},
               "step_tflops_per_gpu": round(tf, 1), "roofline_step_frac": round(tf / step_peak(args.precision)[0], 4),
               "algorithmic_gflop_per_sequence": round(flops / 1e9, 2)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def preembed_image_main(args, dev, world, rank):
    """SURVEY §8(f) row 1, image side: the pre-embedding pass of preprocess_embeddings.py:91-92 —
    Swinv2-base-patch4-window8-256 (the reference's image encoder, train.py:332) over [B,3,256,256]
    images -> [B,64,1024], eval, no grad; a step = `--batch` images (default 64) resident in HBM.
    Each rank embeds its own shard (no collective). Algorithmic work per image (printed): per block
    2 x (12 N C^2 + 4 N L C) FLOP with N tokens, C channels, L = 64 window tokens; per patch merge
    2 x 2 N C^2; patch embedding 2 x 4096 x 48 x 128."""
    from mmfd.swinv2 import Swinv2Config, Swinv2Model, stage_geometry

    B = args.batch
    cfg = Swinv2Config()
    torch.manual_seed(42 + rank)
    m = Swinv2Model(cfg).to(dev).eval().set_precision(args.precision)
    g = torch.Generator(device="cpu").manual_seed(9 + rank)
    px = torch.randn(B, 3, cfg.image_size, cfg.image_size, generator=g).to(dev)
    with torch.no_grad():
        for _ in range(args.warmup):
            m(px)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            m(px)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    if rank == 0:
        R0 = cfg.image_size // cfg.patch_size
        flops = 2 * R0 * R0 * 3 * cfg.patch_size ** 2 * cfg.embed_dim
        geo = stage_geometry(cfg)
        for i, (R, C, H, blocks) in enumerate(geo):
            N = R * R
            for ws, _ in blocks:
                flops += 2 * (12 * N * C * C + 4 * N * ws * ws * C)
            if i < len(geo) - 1:
                flops += 2 * 2 * N * C * C
        imgs = B * world * args.steps / elapsed
        tf = imgs / world * flops / 1e12
        out = {"metric": "images/sec embedded (Swinv2-base-patch4-window8-256, pre-embedding pass)",
               "value": round(imgs, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
               "data": "synthetic N(0,1) pixels [B,3,256,256], random-init weights",
               "config": {"workload": "pre-embedding image pass (SURVEY 8f row 1): swinv2-base forward",
                          "global_batch": B * world, "image_size": cfg.image_size, "parallelism": f"shard{world}"},
               "step_tflops_per_gpu": round(tf, 1), "roofline_step_frac": round(tf / step_peak(args.precision)[0], 4),
               "algorithmic_gflop_per_image": round(flops / 1e9, 2)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    global torch, dist
    import torch
    import torch.distributed as dist
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--precision", choices=["bf16", "fp32"], default=None,
                    help="train: fp32 (default; the reference's arithmetic, bf16 reported beside it); other workloads: bf16")
    ap.add_argument("--mode", choices=["finetune", "frozen"], default="finetune")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=["train", "forward", "extract", "retrieve", "preprocess", "latency",
                                                  "preembed", "preembed_image"],
                    default="train")
    ap.add_argument("--no-bf16", action="store_true", help="skip the secondary bf16 leg of the fp32 headline")
    ap.add_argument("--no-graph", action="store_true",
                    help="time eager steps instead of HIP-graph replays of the captured step (N = 1)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if args.precision is None:  # the reference's fp32 for the training step and the corpus build
        args.precision = "fp32" if args.workload in ("train", "extract") else "bf16"

    import mmfd  # noqa: F401
    from mmfd import kernels as K

    K.load()
    if args.workload == "extract":
        return extract_main(args, dev, world, rank)
    if args.workload == "retrieve":
        return retrieve_main(args, dev, world, rank)
    if args.workload == "forward":
        return forward_main(args, dev, world, rank)
    if args.workload == "preprocess":
        return preprocess_main(args, dev, world, rank)
    if args.workload == "latency":
        return latency_main(args, dev, world, rank)
    if args.workload == "preembed_image":
        if args.batch == 256:
            args.batch = 64
        return preembed_image_main(args, dev, world, rank)
    if args.workload == "preembed":
        if args.batch == 256:
            args.batch = 64
        return preembed_main(args, dev, world, rank)
    res = train_leg(args, dev, world, rank, args.precision)
    log(f"{args.precision} leg: {res['pairs']:.1f} pairs/s")
    sec = None
    if args.precision == "fp32" and not args.no_bf16:
        torch.cuda.empty_cache()
        sec = train_leg(args, dev, world, rank, "bf16")
        log(f"bf16 leg: {sec['pairs']:.1f} pairs/s")
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(res["pairs"], 2), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(res["ms"], 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.precision, "data": "synthetic (Factify-shaped pairs, random-init weights)",
            "config": {"workload": ("full fine-tune " if args.mode == "finetune" else "frozen-encoder ") +
                       "bert-base-uncased + ViT-B/16 + fusion head (768/768, E=256, H=8), fwd+bwd+AdamW",
                       "global_batch": args.batch * world, "seq_len": 128, "image_size": 224,
                       "parallelism": f"dp{world}"},
            "roofline": res["roofline"], "step_launch": res["launch"],
            "step_tflops_per_gpu": round(res["step_tflops"], 1),
            "roofline_step_frac": round(res["step_tflops"] / res["step_peak"][0], 4),
            "roofline_step_peak": {"peak": round(res["step_peak"][0], 1), "unit": "TFLOP/s", "note":
                                   res["step_peak"][1] + f"; step FLOPs = {GFLOP_PER_PAIR[args.mode]} GFLOP/pair "
                                   "(SURVEY 8(d), algorithmic)"},
            "gemm_ms_per_step": res["gemm_ms"], "gemm_tflops_all_shapes": res["gemm_tf"],
            "gemm_kernels": res["gemm_kinds"], "final_loss": res["loss"], "first_step_loss": res["first_loss"],
            "dp_check": res["dp_check"],
            "peak_memory_gb": res["peak_memory_gb"], "memory": res["memory"],
            "fp32_gemm": ("split operands: x = hi + mid + lo bf16 planes staged together per 32-deep K-step, the six "
                          "bf16 MFMA products per fp32 product accumulated directly into the fp32 accumulator, small "
                          "first (error 0.62-1.14x the fp32 MFMA's, bound 1.5x in tests/test_kernels_gpu.py; "
                          "MMFD_FP32_GEMM=native selects the fp32 MFMA)" if K.fp32_gemm_mode() == 1
                          else "fp32 MFMA (v_mfma_f32_16x16x4f32)"),
        }
        if sec is not None:
            out["bf16"] = {"value": round(sec["pairs"], 2), "unit": "pairs/s", "ms_per_step": round(sec["ms"], 3),
                           "step_tflops_per_gpu": round(sec["step_tflops"], 1),
                           "roofline_step_frac": round(sec["step_tflops"] / sec["step_peak"][0], 4),
                           "roofline": sec["roofline"], "final_loss": sec["loss"],
                           "note": "secondary: bf16 MFMA operands, fp32 accumulation / master weights / optimizer"}
        if not args.no_cpu_baseline and world == 1:
            try:
                out["cpu_baseline"], out["parity"] = cpu_baseline(dev)
            except Exception as e:  # the baseline must never hide the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        fx = first_step_parity(args, res)
        if fx is not None:
            out.setdefault("parity", {})["first_step_vs_oracle"] = fx
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def train_leg(args, dev, world, rank, precision):
    """`--warmup` untimed + `--steps` timed training steps of one precision; returns the numbers."""
    from mmfd import kernels as K
    from mmfd.dataset import synthetic_batch
    from mmfd.train import build_flagship

    dp = None
    if world > 1:
        from mmfd.dp import GradAllReduce
        dp = GradAllReduce()
    tr = build_flagship(dev, precision, freeze_encoders=args.mode == "frozen", dp=dp, seed=42, rank=rank)
    batch = synthetic_batch(args.batch, seed=1000 + rank, device=dev)

    # the whole step as one HIP graph. With N > 1 the eager DP step is the default (MMFD_DP_GRAPH=1
    # captures the RCCL gradient all-reduce into the graph as well: deterministic since round 5 —
    # dedicated capture group + thread-local capture mode, mmfd.dp — and self-checked below, but not
    # yet run on a multi-GPU node)
    dp_graph = os.environ.get("MMFD_DP_GRAPH", "0") == "1"
    graphed = not args.no_graph and (world == 1 or dp_graph)
    probe = K.GemmProbe()
    torch.cuda.reset_peak_memory_stats(dev)
    reserved0 = torch.cuda.memory_reserved(dev)
    first_loss = None
    dp_check = None
    if graphed and world > 1:  # capture on every rank, agree, self-check (mmfd.train.capture_dp_step)
        from mmfd.train import capture_dp_step
        graphed, dp_check = capture_dp_step(tr, batch, max(1, args.warmup), dev, log=lambda m: log(f"rank {rank}: {m}"))
        first_loss = getattr(tr, "first_loss", None)
    elif graphed:  # (capture runs its own eager warmup steps first)
        tr.capture(batch, warmup=max(1, args.warmup))
        first_loss = tr.first_loss
    if graphed:
        for _ in range(args.warmup):
            tr.replay()
    else:
        for i in range(args.warmup):
            loss = tr.step(batch)
            if first_loss is None:
                first_loss = loss.clone()
        if world > 1:  # the same cross-rank checksum on the eager DP step
            chk = "eager all-reduce verified" if tr.dp.consistent(tr.dp_state()) else "eager all-reduce MISMATCH"
            dp_check = chk if dp_check is None else f"{dp_check}; {chk}"
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # optimizer steps this trainer has taken when the timed region ends (the last one's loss is
    # final_loss): capture's eager warm-up + warm-up replays + timed replays, or eager warm-up + timed
    opt_steps = (max(1, args.warmup) + args.warmup + args.steps) if graphed else (args.warmup + args.steps)
    if graphed and world > 1:
        opt_steps += 1  # capture_dp_step's verifying replay
    t0 = time.perf_counter()
    if graphed:
        for _ in range(args.steps):
            loss = tr.replay()
    else:
        for _ in range(args.steps):
            loss = tr.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # device memory: the high-water mark of allocated tensors (set by the eager steps before the
    # capture: the graph replays run in the pool the capture reserved), and the reserved growth
    # across capture + replays (the eager steps' cached blocks plus the graph's private pool);
    # tools/mem_account.py separates resident / saved-for-backward / planes / graph pool
    peak_gb = torch.cuda.max_memory_allocated(dev) / 2**30
    mem = {"peak_allocated_gb": round(peak_gb, 1),
           "reserved_gb": round(torch.cuda.memory_reserved(dev) / 2**30, 1),
           "reserved_growth_gb": round((torch.cuda.memory_reserved(dev) - reserved0) / 2**30, 1),
           "breakdown": "profiles/r04_memory.json (tools/mem_account.py)"}
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    ms = 1000.0 * elapsed / args.steps
    pairs = args.batch * world * args.steps / elapsed
    loss_val = loss[0].item()
    log(f"{precision} timed: {pairs:.1f} pairs/s, {ms:.1f} ms/step")

    # per-GEMM device times from two more eager steps of the same trainer after the timed region
    # (events cannot be timed inside a graph), with the two encoders on ONE stream: in the timed
    # step they overlap on two streams, which is faster overall but stretches each kernel's
    # duration by the CUs the other stream holds — the roofline is a property of the kernel alone
    steps_in_prof = 2
    conc, tr.concurrent = tr.concurrent, False
    # (the fusion head's claim-text / claim-image halves likewise on one stream, fusion._two_streams)
    serial_head = os.environ.get("MMFD_SERIAL_HEAD")
    os.environ["MMFD_SERIAL_HEAD"] = "1"
    if graphed:  # the graph's private pool would double the eager probe's footprint
        tr.release_graph()
    # one untimed eager step first: it refills the caching allocator (the hipMallocs of a cold pool
    # would otherwise sit between the probe's events and inflate the first step's GEMM times)
    tr.step(batch)
    torch.cuda.synchronize()
    with probe:
        for _ in range(steps_in_prof):
            tr.step(batch)
    tr.concurrent = conc
    if serial_head is None:
        del os.environ["MMFD_SERIAL_HEAD"]
    else:
        os.environ["MMFD_SERIAL_HEAD"] = serial_head
    prof = probe.summary()
    dom_name, d = max(((k, v) for k, v in prof.items() if "split-K" not in k), key=lambda kv: kv[1]["ms"])
    # achieved = algorithmic FLOPs (2MNK per launch) / measured launch time. The split-operand fp32
    # GEMM (gemm_x6f.hip; gemm.hip X6) runs each fp32 product as six bf16 MFMA products, so its
    # ceiling is the bf16 dense MFMA peak / 6 (= 419.4 TFLOP/s of fp32 products), not the fp32 MFMA peak
    achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
    x6 = "_x6f" in dom_name or dom_name.rstrip().endswith("true>")
    peak = PEAK_TFLOPS[precision] if not x6 else PEAK_TFLOPS["bf16"] / 6
    gemm_ms = sum(v["ms"] for v in prof.values()) / steps_in_prof
    gemm_tf = sum(v["flops"] for v in prof.values()) / (sum(v["ms"] for v in prof.values()) * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic(dom_name)
    kinds = {k: {"launches_per_step": v["launches"] // steps_in_prof, "avg_us": round(1000.0 * v["ms"] / v["launches"], 1),
                 "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1)}
             for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"])}
    tr_conc = conc
    del tr, batch
    roof = {"bound": "mfma", "kernel": dom_name, "achieved": round(achieved, 1), "peak": round(peak, 1),
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
            "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
            "launches_per_step": d["launches"] // steps_in_prof,
            "avg_launch_us": round(1000.0 * d["ms"] / d["launches"], 2),
            "algorithmic_flops_per_launch": int(d["flops"] // d["launches"])}
    if x6:
        roof["peak_note"] = ("split-operand fp32 ceiling: bf16 dense MFMA peak 2516.6 TFLOP/s / 6 bf16 products per "
                             "fp32 product (mid*mid, hi*lo, lo*hi, hi*mid, mid*hi, hi*hi of x = hi + mid + lo planes); "
                             "achieved = 2MNK per launch / launch time")
        roof["bf16_mfma_view"] = {"achieved": round(6 * achieved, 1), "peak": PEAK_TFLOPS["bf16"],
                                  "note": "the same launches as executed bf16 MFMA FLOPs (6 x 2MNK) over the bf16 peak"}
    # context, not the ceiling the frac is taken against: the bf16 MFMA rate this chip holds with no
    # memory traffic at all (tools/mb/gen_g4loop.py V0, MFMAs only on pseudo-random operands,
    # profiles/r06_g4loop_mb_dma_forms.log: 1,790-2,030 TFLOP/s of 2,516.6 = 0.71-0.81, the clock
    # under MFMA load on random data), and what one 1-KB LDS-DMA / vector-memory instruction costs
    # its wave among MFMAs (V2 / V8 / V9: ~45 cycles, not contention between waves, V5-V7)
    roof["mfma_only_rate_note"] = ("bf16 MFMA-only loop on random operands: 0.71-0.81 of the dense peak "
                                   "(power-limited clock; profiles/r06_g4loop_mb_dma_forms.log V0)")
    return {"pairs": pairs, "ms": ms, "loss": round(loss_val, 4), "loss_exact": loss_val, "gemm_ms": round(gemm_ms, 2), "gemm_kinds": kinds,
            "first_loss": None if first_loss is None else [round(v, 6) for v in first_loss.double().cpu().tolist()],
            "dp_check": dp_check,
            "launch": (("one HIP graph per step (captured fwd + bwd + AdamW" + (" + RCCL gradient all-reduce)" if world > 1
                        else ")") if graphed else "eager kernel launches")
                       + ("; text / image encoders on two streams" if tr_conc else "")
                       + "; GEMM times from 2 eager probe steps after the timed region, encoders serialized"),
            "gemm_tf": round(gemm_tf, 1), "step_tflops": pairs / world * GFLOP_PER_PAIR[args.mode] / 1e3,
            "step_peak": step_peak(precision), "roofline": roof, "peak_memory_gb": round(peak_gb, 1), "memory": mem,
            "opt_steps": opt_steps, "world": world}


def first_step_parity(args, res):
    """The timed workload's first optimizer step against the oracle (tests/golden/config3_bs256_p01.npz,
    made by tests/golden/make_config3_bs256.py --recipe bench from this bench's own recipe: weights
    seed 42, batch seed 1000, dropout 0.1 with the kernels' counter-hash masks): the loss vector
    [total, tt, ti, it, ii] of rank 0's first step, max abs error (bound 1e-3 in
    tests/test_fullsize_gpu.py). fp32, bs = 256, full fine-tune only; None otherwise."""
    if args.precision != "fp32" or args.batch != 256 or args.mode != "finetune" or not res.get("first_loss"):
        return None
    path = os.path.join(ROOT, "tests", "golden", "config3_bs256_p01.npz")
    if not os.path.exists(path):
        return None
    import numpy as np
    with np.load(path) as z:
        want = z["loss"].astype(np.float64)
        traj = z["loss_steps"][:, 0].tolist() if "loss_steps" in z.files else None
    got = np.asarray(res["first_loss"], dtype=np.float64)
    out = {"max_abs_err": float(np.abs(got - want).max()), "got": res["first_loss"],
           "oracle": [round(float(v), 6) for v in want], "bound": 1e-3,
           "fixture": "tests/golden/config3_bs256_p01.npz (oracle, chunked whole-batch dropout masks)"}
    traj_path = os.path.join(ROOT, "tests", "golden", "config3_bs256_p01_traj.npz")
    if (traj is None or len(traj) < 2) and os.path.exists(traj_path):
        with np.load(traj_path) as z:
            traj = z["loss_steps"][:, 0].tolist()
    if traj is not None and len(traj) > 1:
        out["oracle_loss_trajectory"] = [round(float(v), 6) for v in traj]
        # final_loss reproduced: the oracle's loss after the same number of optimizer steps on the
        # same batch (one rank: rank r > 0 trains on another seed)
        n = res.get("opt_steps")
        if n and res.get("world", 1) == 1 and n <= len(traj):
            got = float(res.get("loss_exact", res["loss"]))
            out["final_loss"] = {"step": n, "got": round(got, 6), "oracle": round(float(traj[n - 1]), 6),
                                 "abs_err": abs(got - float(traj[n - 1])), "bound": 5e-3,
                                 "fixture": "tests/golden/config3_bs256_p01_traj.npz"}
    return out


def step_peak(precision):
    """(peak TFLOP/s, note) the whole step's algorithmic FLOPs are measured against: the split-operand
    ceiling when the fp32 GEMMs run on split operands, else the dtype's dense MFMA peak"""
    from mmfd import kernels as K
    if precision == "fp32" and K.fp32_gemm_mode() == 1:
        return PEAK_TFLOPS["bf16"] / 6, "split-operand fp32 ceiling (bf16 dense MFMA peak / 6)"
    return PEAK_TFLOPS[precision], f"{precision} dense MFMA peak"


def spawn_ranks(n):
    """`python bench.py --gpus N` without a torch.distributed launcher: start one rank per GPU via
    torch.distributed.run as a CHILD process (this process has not touched the GPU) and exit with
    its status. Under the driver's own `torch.distributed.run` launch WORLD_SIZE is already set."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


if __name__ == "__main__":
    main()
