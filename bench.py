"""Benchmark: PairedAttention paired-GAN training throughput (img/s) at 512x512,
topography=all (9-ch generator input, 12-ch discriminator input), batch 8 per GPU
(BASELINE.json configs[1]; configs[2] = the same step data-parallel over 8 GPUs).

One "step" = one full iteration of models/model.py:615-651 (G forward, D step + Adam(D),
G step against the updated D + Adam(G), the four logged losses read back) over a synthetic
batch already resident in HBM.  Prints ONE JSON line (rank 0).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 8] [--res 512] [--dist-backend nccl|gloo]
  N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
       or plain `python bench.py --gpus N`: with WORLD_SIZE unset the parent starts the N ranks
       itself (launch_ranks) before anything touches the GPU, relays rank 0's JSON line and
       exits non-zero if any rank fails.  `--dist-backend gloo` lets N ranks share fewer GPUs
       (rank r on device r mod device_count): a functional check of the N-rank path on one GPU,
       not an RCCL / xGMI measurement.

--workload attentiongan | cyclegan times the cycle path instead (SURVEY.md §8(f) row 1,
BASELINE.json configs[3]/[4]): one iteration of models/model.py:677-752 (two generators, the
recreated images through the other generator, two discriminators, both Adam steps, the eight
logged losses read back).  --workload pix2pix times the same paired iteration on the Pix2Pix U-Net-256
+ BatchNorm PatchGAN.  The default (paired) is the headline line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak (spec)
BF16_MFMA_PEAK_TFLOPS = 2500.0    # MI355X_MICROARCH.md: bf16 / fp16 dense MFMA peak (spec)
STEP_GFLOP_PER_IMG_512 = 1593.5   # conv fwd 546.1 + conv bwd 1047.3 GFLOP per image
STEP_GB_PER_IMG_512 = 3.96        # algorithmic conv-operand bytes per image at batch 8
HBM_PEAK_TBS = 8.0                # MI355X_MICROARCH.md: HBM3E peak (spec)


def resblock_conv_flops(batch, res):
    """3x3 s1 256->256 conv over (res/4)^2 pixels: 2*M*N*K per launch."""
    m = batch * (res // 4) ** 2
    return 2.0 * m * 256 * (256 * 9)


def resblock_conv_bytes(batch, res):
    """algorithmic HBM bytes of one resblock forward conv launch: the reflect-padded input read once, the
    pre-split fp16 (h, l) weights, the output written once, and the InstanceNorm statistics partials of
    the epilogue ((mean, M2) per 32 output rows and channel)"""
    hw = res // 4
    return 4.0 * batch * ((hw + 2) ** 2 * 256 + hw * hw * 256 + hw * hw // 32 * 256 * 2) + 2 * 2 * 256 * 2304


def resblock_dgrad_bytes(batch, res):
    """algorithmic HBM bytes of one resblock input-gradient interior launch (executor._dgrad_s1_padded): the
    pre-split conv-output gradient (fp16 h + l = 4 B per element) over its 2-px zero border read once, the
    pre-split flipped weights, the (H x W) interior of the padded-domain gradient written once"""
    hw = res // 4
    return 4.0 * batch * ((hw + 4) ** 2 * 256 + hw * hw * 256) + 2 * 2 * 256 * 2304


def resblock_wgrad_bytes(batch, res):
    """algorithmic HBM bytes of one resblock weight-gradient launch (conv_wgrad_f3_kernel<256,0,3>): the pre-split
    gradient's interior rows and the pre-split input over its reflect border 1 read once, one fp32 256 x 2304
    partial slab per pixel split written (plans.wgrad_splits; fg_wgrad_reduce sums them in its own launch)"""
    from floodgan.plans import wgrad_splits
    hw = res // 4
    splits, _ = wgrad_splits(256, 2304, batch * hw * hw, f3=True)
    return 4.0 * batch * (hw * hw * 256 + (hw + 2) ** 2 * 256) + 4.0 * splits * 256 * 2304


# the three resblock conv kinds the bench times live (KernelTimer tags), with their committed counter passes
# (scripts/gpu_pmc.sh KIND=<conv_one kind> + scripts/pmc_summary.py): fwd = the conv1 / conv2 forward launches
# with the InstanceNorm statistics epilogue; dgrad = the input-gradient interior; wgrad = the weight gradient
RESBLOCK_KINDS = {
    "resblock_conv_fwd": dict(kernel="conv_fwd_f3_kernel<256,256,...,STATS>", bytes=resblock_conv_bytes,
                              pmc=[os.path.join(ROOT, "profiles", "round6", "r6_pmc_resblock_fwd_stats_ps.json")]),
    "resblock_conv_dgrad": dict(kernel="conv_fwd_f3_kernel<256,256,...> (input-gradient interior)",
                                bytes=resblock_dgrad_bytes,
                                pmc=[os.path.join(ROOT, "profiles", "round6", "r6_pmc_resblock_dgrad_ps.json")]),
    "resblock_conv_wgrad": dict(kernel="conv_wgrad_f3_kernel<256,0,3>", bytes=resblock_wgrad_bytes,
                                pmc=[os.path.join(ROOT, "profiles", "round6", "r6_pmc_resblock_wgrad_ps.json")]),
}


def step_roofline(img_s_per_gpu, res, peak_conv):
    """The whole step against its ceilings: the conv math's MFMA roof
    (1593.5 GFLOP per 512^2 image), the exact-fp32 MFMA roof, and HBM (3.96 GB per image)."""
    f = STEP_GFLOP_PER_IMG_512 * (res / 512) ** 2 * 1e9
    b = STEP_GB_PER_IMG_512 * (res / 512) ** 2 * 1e9
    ceil_conv = peak_conv * 1e12 / f
    ceil_fp32 = FP32_MFMA_PEAK_TFLOPS * 1e12 / f
    ceil_hbm = HBM_PEAK_TBS * 1e12 / b
    return {"img_s_per_gpu": round(img_s_per_gpu, 3),
            "ceiling_conv_math_img_s": round(ceil_conv, 1), "frac_conv_math": round(img_s_per_gpu / ceil_conv, 4),
            "ceiling_fp32_mfma_img_s": round(ceil_fp32, 1), "frac_fp32_mfma": round(img_s_per_gpu / ceil_fp32, 4),
            "ceiling_hbm_img_s": round(ceil_hbm, 1), "frac_hbm": round(img_s_per_gpu / ceil_hbm, 4),
            "basis": "SURVEY.md §8(d): 1593.5 GFLOP and 3.96 GB per 512x512 image-step; HBM 8 TB/s; the conv "
                     "math's MFMA roof (f16x3: 2500/3 TFLOP/s) and the exact-fp32 MFMA roof 157.3 TFLOP/s"}


def p2p_conv_layers(res, c_in=9):
    """(name, n_out, k_eff, out_pixels, network, needs_dgrad) of every Pix2Pix conv at res x res:
    k_eff = input channels x taps per output (a ConvTranspose2d 4x4 s2 output pixel sees 2x2 taps)"""
    lv = [(c_in, 64, 3), (64, 128, 64), (128, 256, 128), (256, 512, 256)] + [(512, 512, 512)] * 4
    out = []
    for k in range(1, 9):
        i, inner, outer = lv[k - 1]
        out.append((f"down{k}", inner, i * 16, (res >> k) ** 2, "G", k > 1))
        cin_up = inner if k == 8 else 2 * inner
        out.append((f"up{k}", outer, cin_up * 4, (res >> (k - 1)) ** 2, "G", True))
    h = [res // 2, res // 4, res // 8, res // 8 - 1, res // 8 - 2]
    for name, n, kk, hw in (("model.0", 64, 12 * 16, h[0]), ("model.2", 128, 64 * 16, h[1]),
                            ("model.5", 256, 128 * 16, h[2]), ("model.8", 512, 256 * 16, h[3]),
                            ("model.11", 1, 512 * 16, h[4])):
        out.append((name, n, kk, hw * hw, "D", name != "model.0"))
    return out


def p2p_step_gflop_per_img(res):
    """MAC-count FLOPs of one Pix2Pix training iteration per image (models/model.py:615-646): G forward,
    weight + input gradients; D forward + weight/input gradients on 2N images (D step), forward + input
    gradient on N (G step; model.0's input gradient for the 3 image channels only)"""
    tot = 0.0
    for name, n, kk, px, net, dgrad in p2p_conv_layers(res):
        f = 2.0 * px * n * kk
        if net == "G":
            tot += f * (3 if dgrad else 2)
        else:
            tot += 2 * f * (3 if dgrad else 2) + f * 2 + (0 if dgrad else f * 3 / 12)
    return tot / 1e9


def pmc_traffic(kernel_tag, paths):
    """HBM bytes per launch of a kernel from the committed rocprofv3 counter passes
    (scripts/gpu_pmc.sh + scripts/pmc_summary.py: FETCH_SIZE x2 per the gfx950 correction of
    MI355X_MICROARCH.md, plus WRITE_SIZE) averaged over its launch kinds, or None when a summary is missing or does
    not match the kernel."""
    ss = []
    for path in paths:
        try:
            with open(path) as f:
                ss.append(json.load(f))
        except (OSError, ValueError):
            return None
    if any(s.get("kernel_tag") != kernel_tag or "hbm_bytes" not in s for s in ss):
        return None

    def avg(k):
        v = [s.get(k) for s in ss]
        return None if any(x is None for x in v) else sum(v) / len(v)
    return {"bytes_per_launch": avg("hbm_bytes"), "read": avg("hbm_read_bytes"), "write": avg("hbm_write_bytes"),
            "source": [os.path.relpath(p, ROOT) for p in paths], "l2_hit": avg("l2_hit"),
            "mfma_busy": avg("mfma_busy"), "clock_ghz": avg("clock_ghz"),
            "per_kind": {s.get("kind", str(i)): {k: s.get(k) for k in ("hbm_bytes", "l2_hit", "mfma_busy", "clock_ghz",
                                                                        "launch_s")}
                         for i, s in enumerate(ss)}}


def cgroup_cpu_limit():
    """The CPU bandwidth the job's cgroup grants (cgroup v2 cpu.max "quota period" -> quota / period CPUs, or
    None when unlimited / unreadable), with the raw file content as evidence."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            raw = open(path).read().strip()
        except OSError:
            continue
        quota, _, period = raw.partition(" ")
        cpus = None if quota == "max" else round(int(quota) / int(period or 100000), 2)
        return {"path": path, "raw": raw, "cpus": cpus}
    try:                                   # cgroup v1
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return {"path": "/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "raw": f"{q} {p}", "cpus": None if q < 0 else round(q / p, 2)}
    except (OSError, ValueError):
        return None


def host_cpus():
    """What the host offers: lscpu's sockets x cores per socket (physical cores), logical CPUs, the CPU share
    this process may use (affinity; OMP_NUM_THREADS on the GPU box = the box's share) and the cgroup's CPU
    bandwidth limit (the evidence that the share, not the host, bounds the baseline's threads)."""
    info = {"logical": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_cpu_max": cgroup_cpu_limit(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = dict(line.split(":", 1) for line in out.splitlines() if ":" in line)
        kv = {k.strip(): v.strip() for k, v in kv.items()}
        info["model"] = kv.get("Model name")
        info["physical_cores"] = int(kv.get("Socket(s)", 1)) * int(kv.get("Core(s) per socket", 0)) or None
    except (OSError, ValueError):
        pass
    return info


def cpu_baseline(res, threads, steps=3, workload="paired", batches=(1, 8)):
    """Time the CPU oracle (the reference algorithm restated on PyTorch-CPU, pinned to the
    reference's own train_paired / train_cycle outputs; its speed matches the reference's own
    train_paired within the margin recorded in profiles/round2/oracle_vs_reference_speed.log) on a
    bounded sample: `steps` timed iterations at each batch size (1 warm-up iteration at batch 1)."""
    from oracle import attention_cycle as OC  # the checker / CPU baseline only
    from oracle import paired_attention as O
    from oracle import pix2pix as OP

    torch.set_num_threads(threads)
    st = (O.PairedStepOracle() if workload == "paired" else OP.Pix2PixStepOracle() if workload == "pix2pix"
          else OC.CycleStepOracle(model=workload))
    rates = {}
    for bs in batches:
        g = torch.Generator().manual_seed(4321)
        x = torch.rand((bs, 9, res, res), generator=g) * 2 - 1
        y = torch.rand((bs, 3, res, res), generator=g) * 2 - 1
        if bs == batches[0]:
            st.step(x, y)
        t0 = time.perf_counter()
        for _ in range(steps):
            st.step(x, y)
        rates[bs] = bs * steps / (time.perf_counter() - t0)
    host = host_cpus()
    return {"value": round(rates[batches[-1]], 4), "unit": "img/s", "cores": threads, "kind": "port",
            "by_batch": {str(b): round(v, 4) for b, v in rates.items()}, "host": host,
            "sample": f"{steps} timed iterations at batch " + " and ".join(map(str, batches)) +
                      f" (+1 warm-up) of the CPU oracle {workload} step, {res}x{res}, torch-CPU fp32 with {threads} "
                      f"threads (the job's CPU share: cgroup cpu.max "
                      f"{(host.get('cgroup_cpu_max') or {}).get('raw')}, OMP_NUM_THREADS {host.get('omp_num_threads')}; "
                      f"host: {host.get('physical_cores')} physical cores, {host.get('logical')} logical); value = the "
                      f"batch-{batches[-1]} rate"}


def fp32_math_arm(B, R, dev, x, y, steps=5, warmup=1):
    """The same paired step under the exact-fp32 conv math (FLOODGAN_CONV_MATH=fp32: every conv product on
    v_mfma_f32_32x32x2_f32, fp32 in / fp32 accumulate, as the reference's CPU convolutions compute) on a fresh
    seed-47 model and the same batch: the price of exact fp32 arithmetic next to the f16x3 headline."""
    from floodgan import _lib
    from floodgan.model import Model
    prev = _lib.get_conv_math()
    _lib.set_conv_math("fp32")
    try:
        m = Model(model="PairedAttention", num_epochs=2, topography="all", device=dev)
        for _ in range(warmup):
            m.step_fn(x, y).cpu()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            m.step_fn(x, y).cpu()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    finally:
        _lib.set_conv_math(prev)
    return {"conv_math": "fp32", "steps": steps, "warmup": warmup, "ms_per_step": round(1e3 * el / steps, 3),
            "value": round(B * steps / el, 3), "unit": "img/s",
            "note": "same step, batch and seed on a fresh model; every conv on the exact-fp32 MFMA (157.3 TFLOP/s peak)"}


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception as e:          # noqa: BLE001 - reported, not fatal
        return f"unknown ({type(e).__name__})"


def rccl_world1(args):
    """`--rccl-world1`: execute the RCCL path on a one-GPU box.  A one-rank ProcessGroupNCCL is initialised and
    the step's bucketed asynchronous SUM all-reduces (parallel.FlatGrads: D's before Adam(D), G's overlapping the
    generator backward -- models/model.py:632-633, :645-646) are forced through it although world == 1, where they
    are identities.  Two seed-47 models step on the same batch, one with the collectives forced (arm "rccl") and
    one without ("none"), alternating step by step; the line reports each arm's median step time, the number of
    collectives per step and whether the two arms' losses and final parameters are bit-identical."""
    import statistics

    os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=os.environ.get("MASTER_PORT") or str(_free_port()))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    from floodgan import parallel
    from floodgan.model import Model
    B, R = args.batch, args.res
    g = torch.Generator().manual_seed(1234)
    x = (torch.rand((B, 9, R, R), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((B, 3, R, R), generator=g) * 2 - 1).to(dev)
    arms = {a: Model(model="PairedAttention", num_epochs=2, topography="all", device=dev) for a in ("none", "rccl")}
    calls = {"n": 0}
    real_all_reduce = dist.all_reduce

    def counting_all_reduce(*a, **k):
        calls["n"] += 1
        return real_all_reduce(*a, **k)
    dist.all_reduce = counting_all_reduce
    times = {a: [] for a in arms}
    losses = {a: [] for a in arms}
    try:
        for i in range(args.warmup + args.steps):
            for a, m in arms.items():
                prev = parallel.set_force_collectives(a == "rccl")
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                v = m.step_fn(x, y).cpu()
                torch.cuda.synchronize()
                parallel.set_force_collectives(prev)
                if i >= args.warmup:
                    times[a].append(time.perf_counter() - t0)
                losses[a].append(v)
    finally:
        dist.all_reduce = real_all_reduce
    n_steps = args.warmup + args.steps
    same_losses = all(torch.equal(p, q) for p, q in zip(losses["none"], losses["rccl"]))
    pa = [p for net in (arms["none"].generator, arms["none"].discriminator) for p in net.parameters()]
    pb = [p for net in (arms["rccl"].generator, arms["rccl"].discriminator) for p in net.parameters()]
    same_params = all(torch.equal(p, q) for p, q in zip(pa, pb))
    step = arms["rccl"].step_fn
    med = {a: statistics.median(t) * 1e3 for a, t in times.items()}
    out = {"metric": "rccl_world1", "backend": dist.get_backend(), "world_size": dist.get_world_size(),
           "rccl_version": _rccl_version(),
           "steps": args.steps, "warmup": args.warmup,
           "config": {"workload": f"PairedAttention paired train step, {R}x{R}, topography=all, batch {B}"},
           "collectives_per_step": calls["n"] / n_steps,
           "buckets_per_step": len(step.gflat.buckets) + len(step.dflat.buckets),
           "bytes_per_step": 4 * (step.gflat.flat.numel() + step.dflat.flat.numel()),
           "ms_per_step_none": round(med["none"], 3), "ms_per_step_rccl": round(med["rccl"], 3),
           "overhead_ms": round(med["rccl"] - med["none"], 3),
           "losses_bit_identical": same_losses, "params_bit_identical": same_params,
           "losses_last_step": [round(float(v), 5) for v in losses["rccl"][-1]]}
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    return 0 if (same_losses and same_params and calls["n"] == n_steps * out["buckets_per_step"]) else 1


def rank_envs(n, port, base=None, backend="nccl"):
    """The environments of the N ranks `launch_ranks` starts: what torch.distributed.run would set
    (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR / MASTER_PORT on 127.0.0.1) plus the
    backend, over a copy of `base` (os.environ by default; HSA_ENABLE_IPC_MODE_LEGACY=0 is kept)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLOODGAN_DIST_BACKEND=backend)
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        envs.append(e)
    return envs


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, backend="nccl", script=None, timeout=None):
    """Start N rank processes of this script (one per GPU) and wait for them.  Called before any
    GPU call in the parent, so the children are fresh processes (never an exec of a GPU process).
    Rank 0's stdout (the JSON line) is relayed to our stdout; the other ranks' stdout goes to our
    stderr.  When a rank fails the others are terminated (they would block in a collective) and
    the first non-zero exit code is returned."""
    import subprocess
    import threading
    script = script or os.path.abspath(__file__)
    procs = []
    for env in rank_envs(n, _free_port(), backend=backend):
        out = subprocess.PIPE if env["RANK"] == "0" else sys.stderr
        procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env, stdout=out,
                                      text=True if out is subprocess.PIPE else None))

    def relay(stream):
        for line in stream:
            sys.stdout.write(line)
            sys.stdout.flush()
    th = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    th.start()
    t0, rc = time.time(), 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad or (timeout is not None and time.time() - t0 > timeout):
            rc = bad[0] if bad else 124
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.2)
    th.join(timeout=10)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default=None,
                    help="process-group backend for N > 1 (default nccl = RCCL; gloo lets N ranks share one GPU)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="images per GPU")
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32-math", action="store_true",
                    help="skip the fp32_math sub-record (5 steps of the same step under the exact-fp32 conv math)")
    ap.add_argument("--timeout", type=float, default=0,
                    help="N > 1 self-launch: seconds before hung ranks are terminated (rc 124); 0 = 900 + 30 s per step")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--workload", choices=["paired", "pix2pix", "attentiongan", "cyclegan"], default="paired")
    ap.add_argument("--data", choices=["resident", "tiles"], default="resident",
                    help="tiles: feed the step through the staged tile pipeline (floodgan.data.TileLoader) from "
                         "synthetic TIFF tiles on disk, --res = Resize size, --crop quadrants (BASELINE configs[4])")
    ap.add_argument("--dropout-rng", choices=["device", "host"], default="host",
                    help="pix2pix: Dropout(0.5) masks = torch's CPU stream, exactly as the reference's CPU path draws "
                         "them, regenerated on the device (host: the default, RNG parity) or hashed on the device "
                         "(device: no RNG parity)")
    ap.add_argument("--crop", type=int, default=None)
    ap.add_argument("--tile", type=int, default=1024, help="raw tile edge for --data tiles (xBD tiles are 1024)")
    ap.add_argument("--tiles", type=int, default=8, help="distinct synthetic tiles for --data tiles")
    ap.add_argument("--timer-events", choices=["dispatch", "none", "device", "system"], default="dispatch",
                    help="how ops.KernelTimer times the tagged kernels: events on the kernel's own dispatch packet "
                         "(default), or marker events around the call with no / device / system release ('system' "
                         "is torch.cuda.Event's, ~6 us of L2 writeback per event inside the timed step)")
    ap.add_argument("--rccl-world1", action="store_true",
                    help="execute the step's bucketed RCCL all-reduces in a one-rank process group (identities) "
                         "beside the same step without them: overhead and bit-identity (one-GPU evidence of the "
                         "RCCL path; not a scaling measurement)")
    args = ap.parse_args()
    if args.rccl_world1:
        if args.gpus != 1 or "WORLD_SIZE" in os.environ and os.environ["WORLD_SIZE"] != "1":
            sys.exit("bench.py --rccl-world1 runs one rank")
        sys.exit(rccl_world1(args))

    backend = args.dist_backend or os.environ.get("FLOODGAN_DIST_BACKEND", "nccl")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # nothing has touched the GPU yet: start the N ranks as children and relay rank 0's line; ranks that
        # hang (a collective that never completes) are terminated after a generous limit, rc 124
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], backend=backend,
                              timeout=args.timeout or 900 + 30 * (args.steps + args.warmup)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a "
                 f"{world}-rank run as {args.gpus} GPUs")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()               # counting devices does not initialise the GPU
    if world > 1 and backend == "nccl" and ndev < int(os.environ.get("LOCAL_WORLD_SIZE", world)):
        sys.exit(f"bench.py: {world} RCCL ranks need one GPU each, {ndev} visible (use --dist-backend gloo "
                 f"to share)")
    local_dev = local % max(ndev, 1)
    if world > 1:
        torch.cuda.set_device(local_dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local_dev)

    from floodgan import _lib, ops
    from floodgan.model import Model
    from floodgan.parallel import broadcast_params

    B, R = args.batch, args.res
    cycle = args.workload in ("attentiongan", "cyclegan")
    p2p = args.workload == "pix2pix"
    loader = None
    if args.data == "tiles":
        loader, tmpdir = tile_loader(args, B, rank, world, dev)
        R = R // int(round((args.crop or 1) ** 0.5))       # the model sees the crop windows
    m = Model(model={"paired": "PairedAttention", "pix2pix": "Pix2Pix", "attentiongan": "AttentionGAN",
                     "cyclegan": "CycleGAN"}[args.workload], num_epochs=2, topography="all", device=dev)
    nets = ([m.pre_to_post_generator, m.post_to_pre_generator, m.pre_discriminator, m.post_discriminator] if cycle
            else [m.generator, m.discriminator])
    if p2p:
        m.generator.dropout_rng = args.dropout_rng
    if world > 1:
        for net in nets:
            broadcast_params(net)
    step_fn = m.cycle_step_fn if cycle else m.step_fn
    if loader is None:
        g = torch.Generator().manual_seed(1234 + rank)
        x = (torch.rand((B, 9, R, R), generator=g) * 2 - 1).to(dev)
        y = (torch.rand((B, 3, R, R), generator=g) * 2 - 1).to(dev)

        def step():
            return step_fn(x, y)
    else:
        def batches():
            epoch = 0
            while True:
                torch.manual_seed(epoch)                 # models/model.py:609 / :676
                for xb, yb, _ in loader:
                    yield xb, yb
                epoch += 1
        it = batches()

        def step():
            xb, yb = next(it)
            return step_fn(xb, yb)

    for _ in range(args.warmup):
        step().cpu()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    tag = "p2p_d_model8_fwd" if p2p else "resblock_conv_fwd"
    timer = ops.KernelTimer([tag] + ([] if p2p or cycle else ["resblock_conv_dgrad", "resblock_conv_wgrad"]),
                            events=args.timer_events)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with timer:
        for _ in range(args.steps):
            losses = step().cpu()           # the reference logs the losses every iteration
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    math = _lib.get_conv_math()
    fp32_rec = None
    if world == 1 and not (cycle or p2p) and loader is None and not args.no_fp32_math and math != "fp32":
        fp32_rec = fp32_math_arm(B, R, dev, x, y)
    # split maths execute several 16-bit MFMA products per fp32 multiply-add: the roof for fp32
    # work is the 16-bit dense MFMA peak / products (the fp32 MFMA path's roof is 157.3)
    nprod = {"f16x3": 3, "fwd_f16x3": 3, "bf16x6": 6, "fwd_x6": 6}.get(math)
    peak = BF16_MFMA_PEAK_TFLOPS / nprod if nprod else FP32_MFMA_PEAK_TFLOPS
    fwd_x6 = nprod is not None
    all_durs = timer.durations_ms()
    durs = all_durs[tag]
    avg_ms = sum(durs) / max(len(durs), 1)
    if p2p:
        # the discriminator's model.8 conv (256 -> 512, 4x4 s1): per step one 2B-image launch (D step) and
        # one B-image launch (G step) -> average B * 1.5 images per launch
        hw = R // 8 - 1
        flops = 2.0 * (1.5 * B) * hw * hw * 512 * (256 * 16)
    else:
        flops = resblock_conv_flops(B, R)
    achieved = flops / (avg_ms * 1e-3) / 1e12

    if rank == 0:
        img_s = world * B * args.steps / elapsed
        out = {
            "metric": ("GAN training images/sec (512x512, PairedAttention)" if not (cycle or p2p) else
                       f"GAN training images/sec ({R}x{R}, {m.model} cycle)" if cycle else
                       f"GAN training images/sec ({R}x{R}, Pix2Pix)"),
            "value": round(img_s, 3),
            "unit": "img/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic U[-1,1) tiles resident in HBM, seed-47 weights (models/model.py:80)" if loader is None
                     else f"synthetic {args.tile}x{args.tile} TIFF tiles ({args.tiles} distinct, 9-ch float32 inputs + "
                          f"3-ch targets) decoded, staged (pinned ring + copy stream) and transformed (Resize {args.res}, "
                          f"crop={args.crop}, fliplr versions) by floodgan.data.TileLoader inside the timed region"),
            "config": {"workload": (f"PairedAttention paired train step, {R}x{R}, topography=all "
                                    f"(9-ch G input, 12-ch D input), batch {B}/GPU" if not (cycle or p2p) else
                                    f"Pix2Pix paired train step (U-Net-256 G with BatchNorm + Dropout, BatchNorm "
                                    f"PatchGAN), {R}x{R}, topography=all, batch {B}/GPU, dropout masks "
                                    f"{'= torch CPU-generator stream as the reference draws them, generated on the device (RNG parity)' if args.dropout_rng == 'host' else 'hashed on the device (no RNG parity)'}"
                                    if p2p else
                                    f"{m.model} train_cycle step (2 G + 2 D, recreated images, Adam x2), {R}x{R}, "
                                    f"topography=all (9-ch G and D inputs), batch {B}/GPU"),
                       "global_batch": world * B, "per_gpu_batch": B, "resolution": R,
                       "parallelism": f"dp{world}"},
            "conv_math": math,
            "roofline": {"bound": "mfma",
                         "kernel": ("conv_fwd_f3_kernel<256,256,...,STATS> (LDS-DMA ring, 8 waves of 64x128, 16x16x32 "
                                    "f16 MFMA on FG_PRESPLIT operands, InstanceNorm statistics epilogue)"
                                    if nprod == 3 else
                                    f"conv_fwd_x6_kernel<MathBF16x6,128,256,64,64>" if fwd_x6 else
                                    "conv_fwd_kernel<128,128,64,64>") + (
                                        f" Pix2Pix D model.8 4x4 s1 256->512 @{R // 8 - 1}x{R // 8 - 1}" if p2p else
                                        " resblock 3x3 256->256 @128x128"),
                         "achieved": round(achieved, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
                         "peak_basis": (f"16-bit dense MFMA 2500 TFLOP/s / {nprod} split products per fp32 MAC"
                                        if fwd_x6 else "fp32 MFMA dense peak"),
                         "frac": round(achieved / peak, 4),
                         "traffic": (None if p2p else
                                     pmc_traffic("conv_fwd_f3_kernel<256,256,...,STATS>" if nprod == 3 else None,
                                                 RESBLOCK_KINDS[tag]["pmc"])),
                         "avg_launch_ms": round(avg_ms, 4), "launches": len(durs),
                         "timing": ("HIP events on the dispatch packet of every tagged launch of the timed steps (hipExtLaunchKernel)"
                                    if args.timer_events == "dispatch" else
                                    f"HIP marker events around every tagged launch of the timed steps "
                                    f"(release: {args.timer_events})"),
                         "flop_per_launch": flops},
            "step_tflops": (None if cycle else
                            round((p2p_step_gflop_per_img(R) if p2p else STEP_GFLOP_PER_IMG_512 * (R / 512) ** 2)
                                  * world * B * args.steps / elapsed / 1e3, 2)),
            "step_roofline": (None if cycle or p2p else step_roofline(img_s / world, R, peak)),
            "losses_last_step": [round(float(v), 5) for v in losses],
        }
        tr = out["roofline"]["traffic"]
        if p2p:
            gf = p2p_step_gflop_per_img(R)
            out["step_roofline"] = {"gflop_per_img": round(gf, 2),
                                    "ceiling_conv_math_img_s": round(peak * 1e3 / gf, 1),
                                    "frac_conv_math": round(img_s / world / (peak * 1e3 / gf), 4),
                                    "basis": "bench.p2p_step_gflop_per_img: MAC FLOPs of every conv of the step"}
        if tr:
            tr["over_algorithmic"] = round(tr["bytes_per_launch"] / resblock_conv_bytes(B, R), 3)
            tr["algorithmic_bytes"] = resblock_conv_bytes(B, R)
        if not (p2p or cycle) and nprod == 3:
            # every resblock conv kind with its own live launch average, fraction and counter pass
            kinds = {}
            for k, spec in RESBLOCK_KINDS.items():
                d = all_durs.get(k) or []
                if not d:
                    continue
                ms = sum(d) / len(d)
                ach = resblock_conv_flops(B, R) / (ms * 1e-3) / 1e12
                alg = spec["bytes"](B, R)
                t = pmc_traffic(spec["kernel"], spec["pmc"])
                if t:
                    t["over_algorithmic"] = round(t["bytes_per_launch"] / alg, 3)
                kinds[k] = {"kernel": spec["kernel"], "achieved": round(ach, 2), "peak": round(peak, 2),
                            "unit": "TFLOP/s", "frac": round(ach / peak, 4), "avg_launch_ms": round(ms, 4),
                            "launches": len(d), "flop_per_launch": resblock_conv_flops(B, R),
                            "algorithmic_bytes": alg, "achieved_algorithmic_GBs": round(alg / (ms * 1e-3) / 1e9, 1),
                            "traffic": t}
            out["roofline"]["per_kind"] = kinds
        if fp32_rec is not None:
            fp32_rec["vs_headline"] = round(fp32_rec["value"] / img_s, 4)
            out["fp32_math"] = fp32_rec
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", 0)) or len(os.sched_getaffinity(0))
            out["cpu_baseline"] = cpu_baseline(R, threads, steps=1 if cycle or p2p else 3, workload=args.workload,
                                               batches=(1,) if cycle or p2p else (1, 8))
        print(json.dumps(out), flush=True)
    if loader is not None:
        import shutil
        shutil.rmtree(tmpdir, ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()


def tile_loader(args, B, rank, world, dev):
    """A synthetic dataset in the reference's on-disk layout (dataset_input/*.tif 9-ch float32,
    dataset_output/*.tif 3-ch float32, metadata/dataset_split.csv; every third tile also listed as its
    'flipped' version) and the staged train loader over it (models/data.py:11-44 -> floodgan.data)."""
    import tempfile

    import numpy as np
    from floodgan.data import create_flood_dataset, write_tile
    root = tempfile.mkdtemp(prefix=f"floodgan_tiles_r{rank}_", dir="/tmp")
    for d in ("dataset_input", "dataset_output", "metadata"):
        os.makedirs(os.path.join(root, d))
    rng = np.random.default_rng(1234 + rank)
    rows = ["image,best_DEM,same_DEM,version,split,disaster,country"]
    for i in range(args.tiles):
        name = f"hurricane-harvey_{i:08d}"
        write_tile(os.path.join(root, "dataset_input", f"{name}_10m.tif"),
                   rng.random((args.tile, args.tile, 9), dtype=np.float32))
        write_tile(os.path.join(root, "dataset_output", f"{name}.tif"),
                   rng.random((args.tile, args.tile, 3), dtype=np.float32))
        rows.append(f"{name},10m,10m,original,train,hurricane-harvey,usa")
        if i % 3 == 0:
            rows.append(f"{name},10m,10m,flipped,train,hurricane-harvey,usa")
    with open(os.path.join(root, "metadata", "dataset_split.csv"), "w") as f:
        f.write("\n".join(rows) + "\n")
    train, _, _ = create_flood_dataset("hurricane-harvey", "same", root, "all", resize=args.res, crop=args.crop,
                                       batch_size=B, csv_path=os.path.join(root, "metadata", "dataset_split.csv"),
                                       device=dev, rank=rank, world=world)
    train.drop_last = True        # fixed batch shape in the timed region
    return train, root


if __name__ == "__main__":
    main()
