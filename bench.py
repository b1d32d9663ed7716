"""Benchmark: frames/s of ORB extract + match at 640x480 (BASELINE.json config 2:
synthetic 640x480 grayscale stream, 1000 features/frame, 8 levels, 1 MI355X),
plus local-BA ms/iter on the 20 KF x 3000 point problem when --lba is on.

A step = one batch of B frames already resident in HBM: ORBextractor::operator()
on every frame (liborbslam2_amd.so, HIP) followed by
ORBmatcher::SearchForInitialization(frame t-1, frame t, window 100, nnratio 0.9,
checkOri) for every consecutive pair.  Multi-GPU: one process per GPU, frames
shard across ranks with no data-path collective (weak scaling); the only
collectives are the timing barrier and the max-over-ranks of the elapsed time.

Prints ONE JSON line on rank 0.
"""
import argparse
import concurrent.futures as cf
import hashlib
import ctypes as C
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pkgload  # noqa: E402

# the OpenMP CPU baselines (oracle_lba_solve_omp, the extraction port) open and close a parallel
# region per loop: keep the worker threads spinning between regions, as a production OpenMP
# build of g2o would be run (read by the system libgomp when the oracle library loads)
os.environ.setdefault("OMP_WAIT_POLICY", "active")

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_TOPS = 78.6            # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md)
# Chip-wide VALU issue rates measured by tools/micro/valu_issue.hip (profiles/r05_valu_issue.txt):
# each workgroup stamps its loop 17 times, so the rate is taken inside the window where every
# workgroup of the launch runs (instructions interpolated from the stamps), beside the wall-clock
# rate; loop bodies of 8, 32 and 128 instructions give the same rate (no fetch limit).  Steady state
# per SIMD: one wave ~5 cycles per wave64 instruction (long bodies), four waves 3.75 (integer VOP3:
# v_perm, v_alignbyte, v_lerp_u8, v_dot4, v_bcnt, v_pk_minimum3_f16, v_xad) / 3.38 (v_fma_f32),
# eight waves 3.23 (v_fma_f32; the integer kernels never had all eight workgroups of a CU resident
# at once, so their 8-wave figure is the wall-clock one, 5.9e11/s).  Chip-wide: integer 6.5e11
# wave-instructions/s = 41.7 T lane-ops/s; v_fma_f32 7.5e11/s = 48.3 T.  Round 4's 33.9 T / 51.5 T
# summed per-workgroup rates over workgroups that were not all running at once (and a loop with
# 3 scalar instructions per 8 VALU); they are superseded.
VALU_MEASURED_TOPS = 41.7        # integer VOP3 issue ceiling (the extraction / matcher kernels' mix)
VALU_MEASURED_F32_TOPS = 48.3    # v_fma_f32 issue ceiling
STAGES = ["resize", "fast_detect", "reserved", "octree", "reserved2", "orient_blur_desc"]
KERNELS = ["k_resize", "k_fast_cell", None, "k_octree", None, "k_orient_desc"]
PMC_TRAFFIC = ROOT / "profiles" / "r06_pmc_traffic.json"   # tools/pmc_run.sh + tools/pmc_traffic.py
PMC_VALU = ROOT / "profiles" / "r06_valu_pmc.json"         # tools/gpu_pmc_all.sh + tools/pmc_valu.py


def pmc_traffic(kernel, W, H, NF, Bs):
    """HBM bytes per bench stage launch from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes.

    PMC counters cannot be read inside the timed run (gpurun forbids mixing them with traces, and
    counter collection serialises dispatches), so they come from a separate profiling pass of this
    same bench configuration; None when that pass does not match the current configuration."""
    try:
        doc = json.loads(PMC_TRAFFIC.read_text())
        cfg = doc["config"]
        if (int(cfg["width"]), int(cfg["height"]), int(cfg["nfeatures"]), int(cfg["frames_per_launch"])) \
                != (W, H, NF, Bs):
            return None
        return int(doc["kernels"][kernel]["traffic_bytes_per_batch"])
    except (OSError, KeyError, ValueError):
        return None


def pmc_valu_ops(kernel, W, H, NF, Bs):
    """VALU lane-ops (SQ_INSTS_VALU x 64) per launch of `kernel` from the committed PMC pass of
    this configuration; None when that pass does not match it."""
    try:
        doc = json.loads(PMC_VALU.read_text())
        cfg = doc["config"]
        if (int(cfg["width"]), int(cfg["height"]), int(cfg["nfeatures"]), int(cfg["frames_per_launch"])) \
                != (W, H, NF, Bs):
            return None
        return float(doc["kernels"][kernel]["valu_lane_ops"])
    except (OSError, KeyError, ValueError):
        return None


PMC_LANES = ROOT / "profiles" / "r06_lanes_pmc.json"   # tools/pmc_run.sh lanes ... + tools/pmc_lanes.py
# rocprofv3 --kernel-trace --stats of the bench's own 128-frame extraction launch run alone on one
# stream (tools/gpu_ext_isolated.sh: bench.py --streams 1 --batch 128), formatted by
# tools/kernel_stats.py; the headline roofline's kernel durations come from it
ISOLATED_STATS = ROOT / "profiles" / "r06_ext_isolated_stats.txt"


def isolated_stats(frames_per_launch=None):
    """{kernel: avg_us} and the header lines of the committed isolated-launch rocprof summary
    (None when absent, or when its `frames_per_launch=` header names another launch size).  Kernel
    names as kernel_stats.py prints them (`void k_fast_cell<40>`)."""
    try:
        lines = ISOLATED_STATS.read_text().splitlines()
    except OSError:
        return None
    if frames_per_launch is not None:
        import re
        fpl = [m.group(1) for ln in lines for m in [re.search(r"frames_per_launch=(\d+)", ln)] if m]
        if not fpl or int(fpl[0]) != int(frames_per_launch):
            return None
    out, head = {}, []
    for ln in lines:
        if "calls=" in ln and "avg_us=" in ln:
            name = ln.split("calls=")[0].strip()
            name = name.replace("void ", "").split("<")[0]
            calls = int(ln.split("calls=")[1].split()[0])
            avg = float(ln.split("avg_us=")[1].split()[0])
            if name not in out or calls > out[name][0]:
                out[name] = (calls, avg)
        elif ln.strip():
            head.append(ln.strip())
    return {"avg_us": {k: v[1] for k, v in out.items()}, "calls": {k: v[0] for k, v in out.items()}, "header": head}


def pmc_lane_util(kernel, W, H, NF, Bs):
    """Active-lane fraction of `kernel`'s VALU instructions (rocprof's VALUUtilization:
    SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64)) from the committed PMC pass; None when
    absent or for another configuration."""
    try:
        doc = json.loads(PMC_LANES.read_text())
        cfg = doc["config"]
        if (int(cfg["width"]), int(cfg["height"]), int(cfg["nfeatures"]), int(cfg["frames_per_launch"])) \
                != (W, H, NF, Bs):
            return None
        return float(doc["kernels"][kernel]["active_lane_frac"])
    except (OSError, KeyError, ValueError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024, help="frames per step per GPU")
    ap.add_argument("--streams", type=int, default=4,
                    help="independent frame sequences per GPU, each on its own HIP stream (batch split)")
    ap.add_argument("--match-stream", action="store_true",
                    help="SearchForInitialization on a second stream per sequence, overlapping the next step's "
                         "extraction (measured slower than the single-stream chain on MI355X)")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--pool", type=int, default=256, help="distinct synthetic frames resident in HBM")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-lba", action="store_true")
    ap.add_argument("--lba-solves", type=int, default=10, help="timed LocalBundleAdjustment calls")
    ap.add_argument("--lba-points", type=int, default=3000)
    ap.add_argument("--lba-kf", type=int, default=20)
    ap.add_argument("--no-lba-scaled", action="store_true", help="skip the 60 KF / 200 KF corridor windows")
    ap.add_argument("--lba-comm", choices=["native", "torch"], default="torch",
                    help="N>1 local BA: one rank per GPU with a torch.distributed (RCCL) all-reduce callback "
                         "(torch, the default), or the library's device-side group driven by rank 0 over every "
                         "rank's device (native: its peer exchange has run on two contexts of one device only, "
                         "so the line marks it unverified on distinct devices)")
    ap.add_argument("--no-stereo", action="store_true", help="skip the config-5 sharded stereo leg")
    ap.add_argument("--stereo-batches", type=int, default=16,
                    help="8-frame EuRoC stereo batches per step of the config-5 leg")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the secondary legs (brute-force 2-NN, stereo config 5, KITTI config 3)")
    return ap.parse_args()


def algorithmic_bytes(stage, lw, lh, n_pre, n_out):
    """Per-frame algorithmic HBM bytes of each stage."""
    P = (lw.astype(np.int64) * lh).tolist()
    if stage == "resize":   # k_pyramid: level 0 read once, levels 1.. written once (fused, LDS-staged)
        return P[0] + sum(P[1:])
    if stage == "fast_detect":
        return sum(P) + 4 * n_pre
    if stage == "octree":
        return 4 * (n_pre + n_out)
    if stage == "orient_blur_desc":
        return n_out * (43 * 43 + 28 + 32)   # raw 43x43 window per keypoint in, keypoint + descriptor out
    raise KeyError(stage)


# Algorithmic op counts ("algorithmic ops"): one op = one arithmetic,
# compare or load on one pixel / sample, counted from the restated algorithm itself, so that
# neither codegen (address arithmetic, compaction, staging) nor idle lanes count as work.
# Packed forms count per pixel (a SWAR compare of 4 pixels = 4 ops, a dot4 = 4 MACs).
ALG_OPS = {
    # FAST pre-test per region pixel: ring 0/4/8/12 and centre loads (5), 4 dark + 4 bright
    # compares, the adjacent-pair test (8 and/or, 1 combine)
    "fast_pixel": 18,
    # per emitted corner (lower bound: every pre-test survivor is scored, only corners counted):
    # 17 loads + 16 differences + the 9-arc min/max (64 for the 3-arcs, 96 for the arcs, 3 final)
    # + NMS (9 loads, 8 max, 2) + emission (5)
    "fast_corner": 17 + 16 + 64 + 96 + 3 + 19 + 5,
    # bilinear resize per output pixel of levels 1..7: 4 loads, 4 MAC, round
    "resize_pixel": 9,
    # octree per pre-octree key: bucket, compare, move (≈ 30)
    "octree_key": 30,
    # per retained keypoint: 43x48 window (516 dword loads, realign, store = 1548), IC_Angle
    # moments (31 rows x 8 dwords x (load + 2 dot4 x 4 + 2) = 2728), horizontal 7-tap pass
    # (43 x 37 outputs x 7 MAC + 4 loads / 4 outputs = 11739), 512 BRIEF samples (rotation 4,
    # round 2, 7 loads, 7 MAC, clamp 2 = 22 each = 11264), 256 compares, atan + sincos (≈60)
    "keypoint": 1548 + 2728 + 11739 + 11264 + 256 + 60,
}


def algorithmic_ops(stage, lw, lh, n_pre, n_out):
    """Per-frame algorithmic ops of a stage (ALG_OPS; n_pre = corners emitted by k_fast_cell,
    n_out = retained keypoints)."""
    lw = lw.astype(np.int64)
    lh = lh.astype(np.int64)
    region = int(np.maximum(lw - 32, 0).dot(np.maximum(lh - 32, 0)))   # [minBorder, w - minBorder)
    if stage == "fast_detect":
        return ALG_OPS["fast_pixel"] * region + ALG_OPS["fast_corner"] * n_pre
    if stage == "resize":
        return ALG_OPS["resize_pixel"] * int((lw[1:] * lh[1:]).sum())
    if stage == "octree":
        return ALG_OPS["octree_key"] * n_pre
    if stage == "orient_blur_desc":
        return ALG_OPS["keypoint"] * n_out
    raise KeyError(stage)


EXT_KERNELS = (("k_pyramid", "resize", 0), ("k_fast_cell", "fast_detect", 1), ("k_octree", "octree", 3),
               ("k_orient_desc", "orient_blur_desc", 5))


def pmc_capture_current():
    """Whether the committed PMC captures (PMC_TRAFFIC / PMC_VALU / PMC_LANES) were taken from the device
    sources in this tree (their provenance hashes, tools/pmc_provenance.py), per file."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_pmc_prov", ROOT / "tools" / "pmc_provenance.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    now = m.provenance()["csrc_sha256"]
    out = {}
    for f in (PMC_TRAFFIC, PMC_VALU, PMC_LANES):
        try:
            out[f.name] = json.loads(f.read_text()).get("provenance", {}).get("csrc_sha256") == now
        except (OSError, ValueError):
            out[f.name] = None
    return out


def measure_copy_peak(dev, mib=1024, reps=8):
    """SURVEY 8d's second HBM denominator: the device-to-device copy rate this GPU sustains (a
    `mib` MiB tensor copied `reps` times on one stream, HIP events around them; read + write bytes
    per copy).  Measured in the run, so a roofline fraction can be read against what a pure
    streaming kernel gets on this box as well as against the 8 TB/s spec."""
    n = mib * (1 << 20) // 4
    src = torch.empty(n, dtype=torch.float32, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize(dev)
    gbs = 2.0 * n * 4 * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return round(gbs, 1)


def extraction_roofline(stage_ms, ncalls, lw, lh, n_pre, n_out, W, H, NF, Bs, iso_ms=None, launches_per_step=1,
                        ms_per_step=None):
    """SURVEY §8d roofline of every extraction kernel, and the dominant one as the line's `roofline`.

    Per kernel two durations: `shared_launch_ms` = the average launch time inside the timed region
    (HIP events on its stream while the other streams' kernels share the chip; a span, not the
    kernel's own duration) and `isolated_launch_ms` = the same 128-frame launch run alone on one
    stream — from the committed rocprofv3 summary ISOLATED_STATS (`isolated_source`), with the
    live HIP-event measurement of this run's isolated pass beside it (`isolated_live_ms`).  The
    fractions use the isolated duration:
      hbm:  achieved = algorithmic bytes per launch (algorithmic_bytes x frames) / duration, peak 8 TB/s;
      valu: achieved = issued lane-ops per launch (SQ_INSTS_VALU x 64, committed PMC pass) /
            duration, peak 78.6 T (nominal), also against the measured 41.7 T integer issue rate.
    The dominant kernel is the one with the largest isolated duration; `bound` is whichever of
    its two fractions (HBM of 8 TB/s, VALU of the measured issue rate) is higher."""
    iso_file = isolated_stats(Bs)
    per = {}
    for name, stage, i in EXT_KERNELS:
        ms = float(stage_ms[i]) / ncalls if ncalls else 0.0
        live = None if iso_ms is None else float(iso_ms[i])
        f_ms = None
        if iso_file and name in iso_file["avg_us"]:
            f_ms = iso_file["avg_us"][name] / 1e3
        dur = f_ms if f_ms else live
        if not dur or dur <= 0:
            continue
        byts = algorithmic_bytes(stage, lw, lh, n_pre, n_out) * Bs
        gbs = byts / (dur * 1e-3) / 1e9
        k = {"isolated_launch_ms": round(dur, 4), "isolated_source": ISOLATED_STATS.name if f_ms else "live HIP events",
             "isolated_live_ms": None if live is None else round(live, 4),
             "live_over_file": None if (live is None or not f_ms) else round(live / f_ms, 3),
             "shared_launch_ms": round(ms, 4) if ms > 0 else None,
             "algorithmic_bytes_per_launch": int(byts), "achieved_gbs": round(gbs, 2),
             "hbm_frac": round(gbs / HBM_PEAK_GBS, 5), "traffic": pmc_traffic(name, W, H, NF, Bs)}
        if k["traffic"]:
            k["traffic_over_algorithmic"] = round(k["traffic"] / byts, 3)
            k["traffic_gbs"] = round(k["traffic"] / (dur * 1e-3) / 1e9, 2)
        alg = algorithmic_ops(stage, lw, lh, n_pre, n_out) * Bs
        k["algorithmic_ops"] = {"ops_per_launch": int(alg), "achieved_tops": round(alg / (dur * 1e-3) / 1e12, 3),
                                "frac": round(alg / (dur * 1e-3) / 1e12 / VALU_PEAK_TOPS, 4)}
        ops = pmc_valu_ops(name, W, H, NF, Bs)
        if ops is not None:
            ach = ops / (dur * 1e-3) / 1e12
            k["valu"] = {"lane_ops_per_launch": ops, "achieved_tops": round(ach, 3), "peak": VALU_PEAK_TOPS,
                         "frac": round(ach / VALU_PEAK_TOPS, 4), "measured_issue_peak": VALU_MEASURED_TOPS,
                         "frac_of_measured_issue_peak": round(ach / VALU_MEASURED_TOPS, 4),
                         "issued_over_algorithmic": round(ops / max(alg, 1), 2),
                         "issue_peak_source": "profiles/r05_valu_issue.txt (all-running window; int VOP3)"}
            util = pmc_lane_util(name, W, H, NF, Bs)
            if util is not None:
                k["valu"]["active_lane_frac"] = util
        per[name] = k
    if not per:
        return None
    dom = max(per, key=lambda n: per[n]["isolated_launch_ms"])
    d = per[dom]
    hbm = {"achieved": d["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": d["hbm_frac"]}
    v = d.get("valu")
    valu = None if v is None else {"achieved": v["achieved_tops"], "peak": VALU_PEAK_TOPS, "unit": "TOP/s",
                                   "frac": v["frac"], "measured_issue_peak": VALU_MEASURED_TOPS,
                                   "frac_of_measured_issue_peak": v["frac_of_measured_issue_peak"]}
    valu_binds = valu is not None and valu["frac_of_measured_issue_peak"] > hbm["frac"]
    head = valu if valu_binds else hbm
    out = {"bound": "valu" if valu_binds else "hbm", "kernel": dom, "achieved": head["achieved"], "peak": head["peak"],
           "unit": head["unit"], "frac": head["frac"], "traffic": d["traffic"],
           "traffic_unit": "bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE, profiles/)",
           "launch_ms": d["isolated_launch_ms"], "launch_ms_source": d["isolated_source"],
           "launch_ms_live_isolated": d["isolated_live_ms"], "live_over_file": d["live_over_file"],
           "frames_per_launch": Bs, "hbm": hbm, "valu": valu,
           "bound_rule": "valu when the kernel's issued lane-ops / isolated duration, as a fraction of the measured "
                         "41.7 T integer issue rate, exceed its algorithmic bytes / isolated duration as a fraction of "
                         "8 TB/s; headline achieved/peak/frac are the binding one's (VALU peak: the nominal 78.6 T)",
           "algorithmic_bytes_per_launch": d["algorithmic_bytes_per_launch"],
           "bytes_model": "SURVEY 8d per kernel: k_pyramid P0 + sum_{l>=1} P_l; k_fast_cell sum_l P_l + 4 N_pre; "
                          "k_octree 4 (N_pre + N); k_orient_desc N (43^2 + 60)",
           "kernels": per}
    if ms_per_step:
        tot = sum(k["isolated_launch_ms"] for k in per.values()) * launches_per_step
        out["isolated_check"] = {"dominant_ms_x_launches_per_step": round(d["isolated_launch_ms"] * launches_per_step, 4),
                                 "four_kernels_ms_x_launches_per_step": round(tot, 4), "ms_per_step": ms_per_step,
                                 "launches_per_step": launches_per_step}
    return out


def progress(rank, msg):
    """A progress line on stderr (rank 0): the timed line stays the only stdout output."""
    if rank == 0:
        print(f"[bench] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


def host_threads():
    """Host threads this process may run on: the lease's CPU share.  The GPU box exports
    OMP_NUM_THREADS (16 per GPU) while its affinity mask shows the whole machine (256 CPUs), so
    the smaller of the two is the share; never the machine's os.cpu_count()."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def host_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    return {"threads_used": host_threads(), "affinity_cpus": aff, "machine_cpus": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_model": model}


def cpu_baseline(frames, nfeatures, budget_s):
    """Oracle (C restatement of the reference, -O2, 1 thread per frame) on a bounded sample."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ref as O
    p = O.params(nfeatures)
    W, H = frames.shape[2], frames.shape[1]
    threads = host_threads()

    def one(i):
        # the sample cycles over the resident frame pool (consecutive pairs stay consecutive)
        return O.extract(p, frames[i % len(frames)])

    # calibrate on 4 frames, then size the sample to the budget
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as pool:
        list(pool.map(one, range(min(4 * threads, len(frames)))))
    t_cal = (time.perf_counter() - t0) / min(4 * threads, len(frames))
    n = int(max(threads, budget_s / max(t_cal, 1e-4)))
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as pool:
        res = list(pool.map(one, range(n + 1)))

        def match(i):
            a, b = res[i], res[i + 1]
            fa = O.FrameView(a["kps"], a["desc"], W, H)
            fb = O.FrameView(b["kps"], b["desc"], W, H)
            prev = np.stack([a["kps"]["x"], a["kps"]["y"]], 1).astype(np.float32).reshape(-1)
            return O.search_for_initialization(fa, fb, prev, nnratio=0.9, window=100)[0]

        list(pool.map(match, range(n)))
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 2), "unit": "frames/s", "cores": threads, "kind": "port", "host": host_info(),
            "sample": f"{n + 1} frames extracted + {n} SearchForInitialization pairs, {W}x{H}, "
                      f"{nfeatures} feat, oracle C restatement, {threads} host threads (1 frame per thread)"}


F64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector and matrix (MI355X_MICROARCH.md)


def lba_roofline(pb, out, world):
    """Per-trial rooflines of the local-BA stages from the profiled pass's HIP-event stage times
    (stage_ms_per_solve / trials):
      * reduced solve (k_ldlt_solve): MFMA f64 flops of the blocked LDL^T's trailing updates,
        8192 per 16x16x16 tile update, T = ceil(6P/16) block columns;
      * Schur complement (k_point_schur + k_schur_pairs): SURVEY 8d's algorithmic
        F_schur = sum_p [40 + 144 k_p + 216 k_p (k_p + 1) / 2] (k_p = free observers), on the
        f64 VALU (sparse: a densified MFMA GEMM would do ~15x the flops);
      * linearisation (k_edge_lin + k_vertex_reduce): SURVEY 8d's E (112 read + 160 written) +
        M 168 bytes against HBM."""
    trials = max(out["trials"], 1)
    st = out["stage_ms_per_solve"]
    fixed = pb["pose_fixed"].astype(bool)
    free_edge = ~fixed[pb["edge_pose"]]
    kp = np.bincount(pb["edge_point"][free_edge], minlength=len(pb["point_xyz"]))
    P = int(np.count_nonzero(~fixed & np.isin(np.arange(len(fixed)), pb["edge_pose"])))
    T = (6 * P + 15) // 16
    tiles = sum((T - k - 1) * (T - k) // 2 for k in range(T))
    mfma_flops = tiles * 8192
    f_schur = float(np.sum(40 + 144 * kp + 216 * kp * (kp + 1) / 2)) / world
    E, M = len(pb["edge_point"]) / world, len(pb["point_xyz"]) / world
    lin_bytes = E * (112 + 160) + M * 168
    t_solve = st["solve_ms"] / trials * 1e-3
    t_schur = st["schur_ms"] / trials * 1e-3
    t_lin = st["linearize_ms"] / trials * 1e-3

    def r(x, n=4):
        return round(x, n)
    return {
        "reduced_solve": {"bound": "mfma", "unit": "TFLOP/s", "flops_per_trial": mfma_flops,
                          "us": r(t_solve * 1e6, 2), "achieved": r(mfma_flops / t_solve / 1e12, 5),
                          "peak": F64_PEAK_TFLOPS, "frac": r(mfma_flops / t_solve / 1e12 / F64_PEAK_TFLOPS, 7),
                          "note": f"n = {6 * P}, {tiles} 16x16 tile updates of 4 v_mfma_f64_16x16x4 each; "
                                  "latency-bound pivot chain on one workgroup"},
        "schur": {"bound": "valu", "unit": "TFLOP/s", "flops_per_trial": int(f_schur), "us": r(t_schur * 1e6, 2),
                  "achieved": r(f_schur / t_schur / 1e12, 5), "peak": F64_PEAK_TFLOPS,
                  "frac": r(f_schur / t_schur / 1e12 / F64_PEAK_TFLOPS, 6)},
        "linearize": {"bound": "hbm", "unit": "GB/s", "bytes_per_iteration": int(lin_bytes), "us": r(t_lin * 1e6, 2),
                      "achieved": r(lin_bytes / t_lin / 1e9, 2), "peak": 8000.0,
                      "frac": r(lin_bytes / t_lin / 1e9 / 8000.0, 6)},
    }


def bench_lba(args, amd, dev, local, rank, world):
    """Local BA (BASELINE.json config 4: 20 KF x 3000 points), landmarks sharded over ranks
    with RCCL all-reduce of the reduced camera system.  ms/iter = wall time of the
    optimisation / LM outer iterations executed (both optimize() rounds)."""
    from orb_slam2_amd import synth
    pb = synth.ba_problem(n_local=args.lba_kf, n_points=args.lba_points)
    nk, ne = len(pb["Tcw"]), len(pb["edge_point"])
    native = world > 1 and args.lba_comm == "native"
    fallback = None
    if native:
        # the drop-in's multi-GPU path: ONE process (rank 0, LocalMapping's thread) drives a group
        # of contexts on all the ranks' devices; the library's peer-to-peer all-reduce over xGMI
        # carries the exchange (lba_group_*); the other ranks wait at the barrier.  Without peer
        # access between the devices the group cannot form: every rank then takes the torch path.
        ndev = torch.cuda.device_count()
        devices = [r % ndev for r in range(world)]
        ok = torch.ones(1, dtype=torch.float64, device=dev)
        ctx = None
        if rank == 0:
            try:
                ctx = amd.LocalBAGroup(devices)
            except RuntimeError as exc:
                fallback = str(exc)
                ok.zero_()
        torch.distributed.broadcast(ok, src=0)
        if ok.item() == 0:
            native = False
            fallback = fallback or "lba_group_create failed on rank 0"
    if not native:
        ctx = amd.LocalBA(local)
        # a dedicated stream (the legacy default stream cannot be captured into the LM slot graph);
        # RCCL calls of the all-reduce callback are issued on the same stream
        stream = torch.cuda.Stream(dev)
        ctx.set_stream(stream.cuda_stream)
    # per-collective cost of the RCCL callback during the timed solves (HIP events on the LM stream
    # around each all_reduce; DESIGN §5's cost model is checked against these at N > 1)
    coll = {"on": False, "ev": [], "calls": 0, "bytes": 0}
    if world > 1 and not native:
        ws = torch.zeros(max(36 * nk * nk + 6 * nk, ne) + 64, dtype=torch.float64, device=dev)

        def ar(off, cnt, op):
            with torch.cuda.stream(stream):
                if coll["on"]:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                torch.distributed.all_reduce(ws[off:off + cnt], op=torch.distributed.ReduceOp.SUM if op == 0
                                             else torch.distributed.ReduceOp.MAX)
                if coll["on"]:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record(stream)
                    coll["ev"].append((e0, e1))
                    coll["calls"] += 1
                    coll["bytes"] += 8 * cnt
        ctx.set_comm(rank, world, ws, ar)
    if native and rank != 0:   # rank 0 runs the sharded solves; its result is broadcast below
        torch.distributed.barrier()
        obj = [None]
        torch.distributed.broadcast_object_list(obj, src=0)
        return obj[0]

    def body():
        nonlocal ctx, fallback
        # warm-up: allocations, code objects and the LM-slot graphs of both group shapes (the
        # first solves instantiate them); LocalMapping calls LocalBundleAdjustment once per keyframe,
        # so the steady state is what it sees
        call = ctx.prepared(pb)
        grp_live = native   # the group's solves are the timed ones (False after a fallback)
        try:
            for _ in range(3):
                call()
        except RuntimeError as exc:
            if not native:
                raise
            # the group failed on this node (e.g. a timed-out exchange): rank 0 times its own device
            # alone and says so; the waiting ranks still get the broadcast below
            fallback = f"lba_group_solve failed: {exc}; rank 0 alone"
            grp_live = False
            ctx = amd.LocalBA(local)
            call = ctx.prepared(pb)
            for _ in range(3):
                call()
        if world > 1 and not native:   # (native: the other ranks wait at the barrier below)
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        iters, times = 0, []
        coll["on"] = True
        for _ in range(args.lba_solves):   # timed: the lba_solve C-ABI call (arguments marshalled once)
            t0 = time.perf_counter()
            its, _, _ = call()
            times.append(time.perf_counter() - t0)
            iters += sum(its)
        coll["on"] = False
        tot = sum(times)
        if grp_live:
            ex_ms, n_ex = ctx.stats()
            r = ctx.solve(pb)
            st = None
            erased = int(np.count_nonzero(r["edge_erase"]))
        elif native:   # (fallback: rank 0's own solve, no stage split)
            r = ctx.solve(pb)
            st = None
            erased = int(np.count_nonzero(r["edge_erase"]))
        else:
            # stage split from a separate profiled pass (per-slot HIP events; kernels enqueued one by
            # one, so these solves are slower than the timed ones above)
            ctx.profile(True)
            for _ in range(args.lba_solves):
                r = ctx.solve(pb)      # (decisions below: the same in every solve of this problem)
            st = ctx.stats()
            ctx.profile(False)
            er = torch.tensor([float(np.count_nonzero(r["edge_erase"]))], dtype=torch.float64, device=dev)
            if world > 1:      # each rank flags the edges of its own landmark shard
                torch.distributed.all_reduce(er)
            erased = int(er.item())
            if world > 1:
                t = torch.tensor([tot], dtype=torch.float64, device=dev)
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
                tot = float(t.item())
        out = {"config": f"{args.lba_kf} KF (+4 fixed) x {args.lba_points} points, {ne} mono edges, "
                         f"landmarks sharded x{world}",
               "ms_per_iter": round(1000 * tot / max(iters, 1), 4),
               "solve_ms": round(1000 * tot / args.lba_solves, 3),
               "iterations_per_solve": iters / args.lba_solves, "trials": r["trials"],
               "n_gpus": world,
               "native_group_unavailable": fallback,
               "collective": ("none" if world == 1 else
                              "library device-side exchange over xGMI (lba_group: flag words + peer reads, one process "
                              "driving every device, slots in HIP graphs; verified before this run on two contexts "
                              "of one device only)" if grp_live else
                              "none (the group failed; rank 0's device alone)" if native else
                              "torch.distributed all_reduce callback (RCCL), one process per GPU"),
               # LM decisions of the last timed solve: identical for every world size (landmark shards
               # only reorder the f64 sums; tests/test_bench_ranks.py compares N=1 with N=2)
               "decisions": {"iterations": [int(x) for x in r["iterations"]], "trials": int(r["trials"]),
                             "chi2_trace": [float(x) for x in r["trace"][:, 1]],
                             "erased_edges": erased}}
        if st is not None:
            out["stage_ms_per_solve"] = {k: round(st[k] / args.lba_solves, 4) for k in
                                         ("linearize_ms", "schur_ms", "solve_ms", "update_ms")}
        if coll["calls"]:
            torch.cuda.synchronize(dev)
            us = [1000.0 * a.elapsed_time(b) for a, b in coll["ev"]]
            out["rccl_callback"] = {
                "collectives_per_solve": round(coll["calls"] / args.lba_solves, 2),
                "us_per_collective_mean": round(float(np.mean(us)), 2),
                "us_per_collective_median": round(float(np.median(us)), 2),
                "bytes_per_collective_mean": round(coll["bytes"] / coll["calls"], 1),
                "collective_share_of_solve": round(sum(us) / 1e6 / max(tot, 1e-12), 4),
                "note": "HIP events on the LM stream around each torch.distributed.all_reduce (RCCL) issued by "
                        "the library's host callback, rank-local, timed solves only"}
        if grp_live:
            # (host-ordered exchange: events around each collective; the device-side default has
            # none — its cost is in the kernel trace as k_grp_sync / k_grp_reduce)
            out["exchange_us_per_collective"] = round(1000 * ex_ms / max(n_ex, 1), 2) if ex_ms > 0 else None
            out["collectives_per_trial"] = round(n_ex / max(1, (3 + args.lba_solves) * r["trials"]), 2)
        if st is not None:   # (the native group's solves have no per-slot stage events)
            out["roofline"] = lba_roofline(pb, out, world)
        if world == 1 and not args.no_cpu:   # the CPU baseline is an N=1 figure
            sys.path.insert(0, str(ROOT / "tests"))
            import oracle_ref as O

            def timed(threads, budget=3.0):
                t0 = time.perf_counter()
                n, it = 0, 0
                while time.perf_counter() - t0 < budget or n < 2:
                    rr = O.lba_solve(pb, threads=threads)
                    it += sum(rr["iterations"])
                    n += 1
                dt = time.perf_counter() - t0
                return dt, n, it
            dt, n, it = timed(None)
            out["cpu_baseline"] = {"ms_per_iter": round(1000 * dt / it, 4), "solve_ms": round(1000 * dt / n, 3),
                                   "cores": 1, "kind": "port", "cpu_model": host_info()["cpu_model"],
                                   "sample": f"{n} LocalBundleAdjustment solves, oracle C restatement of g2o "
                                             f"LM+Schur (dense LDLT), 1 thread (reference builds g2o without OpenMP)"}
            th = host_threads()
            dt, n, it = timed(th)
            out["cpu_baseline_openmp"] = {
                "ms_per_iter": round(1000 * dt / it, 4), "solve_ms": round(1000 * dt / n, 3), "cores": th, "kind": "port",
                "host": host_info(),
                "sample": f"{n} solves, oracle_lba_solve_omp: g2o's G2O_OPENMP loops (computeActiveErrors, buildSystem "
                          f"edges, Schur landmarks) on {th} threads, bitwise identical to the 1-thread oracle"}
            out["speedup_vs_cpu"] = round(out["cpu_baseline"]["ms_per_iter"] / out["ms_per_iter"], 2)
            out["speedup_vs_cpu_openmp"] = round(out["cpu_baseline_openmp"]["ms_per_iter"] / out["ms_per_iter"], 2)
        return out

    try:
        out = body()
    except Exception as exc:   # rank 0 must still reach the ranks waiting at the barrier below
        if not native:
            raise
        out = {"error": f"{type(exc).__name__}: {exc}", "n_gpus": world}
    if native:   # rank 0 -> the waiting ranks
        torch.distributed.barrier()
        torch.distributed.broadcast_object_list([out], src=0)
    return out


def bench_lba_scaled(args, amd, dev, rank, world):
    """SURVEY 8d's scaled local-BA windows (the reduced system beyond the LDS image: the
    multi-workgroup LDL^T and the pair-list Schur complement): corridor windows of 60 KF x 8,000
    and 200 KF x 100,000 points with banded covisibility (synth.ba_problem_corridor).  N > 1:
    rank 0 drives the device group (lba_group) over every rank's device, as bench_lba does.
    At N = 1 the oracle's OpenMP variant is timed beside it on one solve."""
    sizes = ((60, 8000), (200, 100000))
    native = world > 1 and args.lba_comm == "native"
    if native and rank != 0:
        torch.distributed.barrier()
        obj = [None]
        torch.distributed.broadcast_object_list(obj, src=0)
        return obj[0]
    out = {}
    try:
        _lba_scaled_sizes(args, amd, dev, world, native, sizes, out, rank)
    except Exception as exc:   # rank 0 must still reach the ranks waiting at the barrier below
        if not native:
            raise
        out["error"] = f"{type(exc).__name__}: {exc}"
    out["note"] = ("corridor windows, banded covisibility; ms_per_iter = lba_solve wall / LM iterations"
                   + (f"; landmarks sharded over {world} devices by one process (lba_group, unverified on "
                      f"distinct devices before this run)" if native else
                      f"; landmarks sharded over {world} ranks, torch.distributed all_reduce (RCCL) callback, "
                      f"max over ranks" if world > 1 else ""))
    if native:
        torch.distributed.barrier()
        torch.distributed.broadcast_object_list([out], src=0)
    return out


def mw_envelope_mfma_flops(pb):
    """The multi-workgroup LDL^T's MFMA flops per trial inside the reduced matrix's envelope
    (k_mw_envelope / k_ldlt_mw_step): free poses in id order (g2o's block order), pose j's rows
    starting at 6 min{i : poses i, j share a landmark}, per 16-row tile the least start, and per
    32-column panel the trailing tiles (I >= K) whose two tile rows both reach into the panel,
    16 x 16 x 32 multiply-adds each."""
    fixed = pb["pose_fixed"].astype(bool)
    order = [int(i) for i in np.argsort(pb["pose_id"], kind="stable") if not fixed[i]]
    P = len(order)
    if P == 0:
        return 0
    idx = np.full(len(fixed), -1, np.int64)
    idx[order] = np.arange(P)
    pe, pt = idx[np.asarray(pb["edge_pose"])], np.asarray(pb["edge_point"])
    keep = pe >= 0
    mn = np.full(len(pb["point_xyz"]), P, np.int64)
    np.minimum.at(mn, pt[keep], pe[keep])
    fp = np.arange(P)
    np.minimum.at(fp, pe[keep], mn[pt[keep]])
    n = 6 * P
    npad = (n + 31) // 32 * 32
    rows = np.arange(npad)
    rf = np.where(rows < n, 6 * fp[np.minimum(rows, n - 1) // 6], rows)
    tfirst = rf.reshape(-1, 16).min(1)
    flops = 0
    for jb in range(0, npad, 32):
        live = int(np.count_nonzero(tfirst[(jb + 32) // 16:] <= jb + 31))
        flops += live * (live + 1) // 2 * 16384
    return flops


def torch_comm_context(amd, dev, rank, world, nk, ne):
    """A LocalBA context of this rank whose collectives are torch.distributed.all_reduce calls (RCCL
    over xGMI with one process per GPU, gloo when ranks share a device) on its own stream."""
    ctx = amd.LocalBA(dev.index or 0)
    stream = torch.cuda.Stream(dev)
    ctx.set_stream(stream.cuda_stream)
    ws = torch.zeros(max(36 * nk * nk + 6 * nk, ne) + 64, dtype=torch.float64, device=dev)

    def ar(off, cnt, op):
        with torch.cuda.stream(stream):
            torch.distributed.all_reduce(ws[off:off + cnt], op=torch.distributed.ReduceOp.SUM if op == 0
                                         else torch.distributed.ReduceOp.MAX)
    ctx.set_comm(rank, world, ws, ar)
    ctx._keep = (stream, ws)
    return ctx


def _lba_scaled_sizes(args, amd, dev, world, native, sizes, out, rank=0):
    from orb_slam2_amd import synth
    for nl, npts in sizes:
        pb = synth.ba_problem_corridor(n_local=nl, n_fixed=4, n_points=npts)
        group_error = None
        if world > 1 and not native:   # one rank per GPU, RCCL all-reduce callback
            ctx = torch_comm_context(amd, dev, rank, world, len(pb["Tcw"]), len(pb["edge_point"]))
            call = ctx.prepared(pb)
            for _ in range(2):
                call()
            torch.distributed.barrier()
        elif native:
            try:
                ndev = torch.cuda.device_count()
                ctx = amd.LocalBAGroup([r % ndev for r in range(world)])
                call = ctx.prepared(pb)
                for _ in range(2):
                    call()
            except RuntimeError as exc:   # the group cannot form or a sharded solve failed here:
                group_error = str(exc)    # rank 0's device alone, and the line says so
                ctx = amd.LocalBA(dev.index or 0)
                call = ctx.prepared(pb)
                for _ in range(2):
                    call()
        else:
            ctx = amd.LocalBA(dev.index or 0)
            call = ctx.prepared(pb)
            for _ in range(2):
                call()
        times, iters = [], 0
        for _ in range(5):
            t0 = time.perf_counter()
            its, tr, _ = call()
            times.append(time.perf_counter() - t0)
            iters += sum(its)
        if world > 1 and not native:   # the slowest rank's time
            t = torch.tensor([sum(times)], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            times = [float(t[0]) / 5] * 5
        fixed = pb["pose_fixed"].astype(bool)
        P = int(np.count_nonzero(~fixed))
        T = (6 * P + 15) // 16
        tiles = sum((T - k - 1) * (T - k) // 2 for k in range(T))
        env_flops = mw_envelope_mfma_flops(pb)
        key = f"{nl}kf_{npts // 1000}k"
        out[key] = {"keyframes": nl, "fixed": 4, "points": npts, "edges": int(len(pb["edge_point"])),
                    "reduced_order": 6 * P, "ms_per_iter": round(1000 * sum(times) / max(iters, 1), 4),
                    "solve_ms": round(1000 * float(np.median(times)), 3), "iterations_per_solve": iters / 5,
                    "trials_per_solve": tr, "ldlt_mfma_flops_per_trial": env_flops,
                    "ldlt_mfma_flops_dense_per_trial": tiles * 8192}
        if group_error is not None:
            out[key]["native_group_unavailable"] = group_error
        if world == 1:
            # the reduced solve's share from one profiled solve (per-slot events, kernels enqueued one
            # by one): its f64 MFMA rate against the 78.6 TFLOP/s peak.  The MFMA flops are the
            # trailing-update tiles' inside the reduced matrix's envelope (16x16x32 per tile and
            # 32-column panel, what k_ldlt_mw_* multiply; the dense count is beside it); the pivot
            # chain's VALU work is not counted
            ctx.profile(True)
            rp = ctx.solve(pb)
            stp = ctx.stats()
            ctx.profile(False)
            t_tr = stp["solve_ms"] / max(1, rp["trials"]) * 1e-3
            if t_tr > 0:
                ach = env_flops / t_tr / 1e12
                # (what binds is latency: one kernel boundary + one memory round trip + a 32-column
                # recurrence per panel; the MFMA rate is the context figure)
                out[key]["reduced_solve"] = {"bound": "latency", "us_per_trial": round(t_tr * 1e6, 1),
                                             "achieved_tflops": round(ach, 4), "peak": F64_PEAK_TFLOPS,
                                             "frac": round(ach / F64_PEAK_TFLOPS, 5),
                                             "source": "one profiled solve (stage events; kernels enqueued one by one)"}
        if world == 1 and not args.no_cpu:
            sys.path.insert(0, str(ROOT / "tests"))
            import oracle_ref as O
            th = host_threads()
            t0 = time.perf_counter()
            rr = O.lba_solve(pb, threads=th)
            dt = time.perf_counter() - t0
            out[key]["cpu_baseline_openmp"] = {"ms_per_iter": round(1000 * dt / sum(rr["iterations"]), 3),
                                               "cores": th, "kind": "port", "cpu_model": host_info()["cpu_model"],
                                               "sample": "one LocalBundleAdjustment solve, oracle_lba_solve_omp"}
            out[key]["speedup_vs_cpu_openmp"] = round(out[key]["cpu_baseline_openmp"]["ms_per_iter"] /
                                                      out[key]["ms_per_iter"], 1)
        del ctx


def batch_status(ex=None, m=None, what="leg"):
    """The overflow bits of an extractor's / matcher's batched calls (orb_extractor_batch_status,
    orb_matcher_batch_status; waits for their streams, reading the matcher's clears it).  A set
    bit means some frame's keypoints or some pair's candidate list were truncated, i.e. the leg did
    not compute the reference's result: fail loudly instead of reporting its rate."""
    from orb_slam2_amd import _abi
    lib = _abi.lib()
    es, ms = C.c_int32(0), C.c_int32(0)
    if ex is not None:
        lib.orb_extractor_batch_status(ex._h, C.byref(es))
    if m is not None:
        lib.orb_matcher_batch_status(m._h, C.byref(ms))
    if es.value or ms.value:
        raise SystemExit(f"bench {what}: overflow status extractor={es.value} matcher={ms.value}")
    return {"extractor": es.value, "matcher": ms.value}


def _extract_leg(amd, dev, frames, nf, steps, warmup, pairs_fn=None, matcher=None):
    """Times batched extraction of an HBM-resident frame array (one step = all frames)
    plus an optional per-step device function; returns (seconds per step, buffers).  The
    extractor's overflow bits are read after the timed steps (batch_status)."""
    from orb_slam2_amd import _abi
    B, H, W = frames.shape
    ex = amd.ORBextractor(nf, 1.2, 8, 20, 7, device=dev.index or 0, max_w=W, max_h=H, max_batch=B)
    cap = C.c_int()
    _abi.check("geom", _abi.lib().orb_extractor_geometry(ex._h, W, H, None, None, None, C.byref(cap)))
    cap = cap.value
    imgs = torch.from_numpy(frames).to(dev)
    kps = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    lib = _abi.lib()
    buf = dict(ex=ex, cap=cap, kps=kps, desc=desc, cnt=cnt, stream=st, lib=lib, matcher=matcher)

    def step():
        _abi.check("x", lib.orb_extract_batch_device(ex._h, C.c_void_p(imgs.data_ptr()), H * W, B, W, H,
                                                      C.c_void_p(kps.data_ptr()), C.c_void_p(desc.data_ptr()), cap,
                                                      C.c_void_p(cnt.data_ptr()), C.c_void_p(st)))
        if pairs_fn is not None:
            pairs_fn(buf)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    buf["status"] = batch_status(ex, buf.get("matcher"), "extraction leg")
    return dt, buf


def _camera(name):
    """The reference's YAML camera settings (synth.CAMERAS, pinned to the YAMLs by
    tests/test_reference_data.py); synth.py is loaded on its own, so no HIP library loads here."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_orb_synth_cams", ROOT / "orb-slam2-_amd" / "synth.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.CAMERAS[name]


# Camera.bf as Tracking reads it into the float mbf (R/Examples/Stereo/EuRoC.yaml:25, R/src/Tracking.cpp:95)
EUROC_MBF = float(np.float32(_camera("EUROC")["bf"]))


def _timed_ranks(fn, steps, warmup, dev, world):
    """warmup untimed calls, then `steps` timed ones bracketed by barrier + synchronize on both
    sides; returns the max over ranks of the elapsed seconds."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def bench_config5(args, amd, dev, rank, world):
    """BASELINE config 5: EuRoC-geometry stereo (752x480, 1200 feat, 8 levels), 8-frame batches
    sharded over the ranks (rank r takes its contiguous share of each batch's 8 stereo pairs; no
    data-path collective).  Per pair: ORBextractor on the left and the right image (both kept in
    the two-extractor roles of R/src/Frame.cpp:86-89) and Frame::ComputeStereoMatches
    (R/src/Frame.cpp:551-770) on the device pyramids.  Two timings:
      * throughput: `--stereo-batches` batches per step (strong scaling: the total is fixed);
      * latency: one 8-frame batch per step, sharded the same way (ms per batch, max over ranks)."""
    from orb_slam2_amd import synth
    W, H, NF, PB = 752, 480, 1200, 8
    shard = np.array_split(np.arange(PB), world)[rank]
    cv = synth.canvas(0x5EED0005, W, H)
    out = {"config": f"synthetic EuRoC MH_01 geometry {W}x{H} stereo (smooth integer disparity 5..60 px), {NF} feat, "
                     f"8 levels, mbf {EUROC_MBF}, mb 0 (reference call order); {PB}-frame batches sharded over "
                     f"{world} rank(s)", "pairs_per_batch": PB, "scaling": "strong"}
    for tag, nb in (("throughput", args.stereo_batches), ("latency_one_batch", 1)):
        pairs = [b * PB + int(j) for b in range(nb) for j in shard]
        P = len(pairs)
        step, o = config5_shard(amd, dev, cv, pairs)
        ur, dep, ns, cnt, cap, ex = o["ur"], o["dep"], o["ns"], o["cnt"], o["cap"], o["ex"]
        steps = max(args.steps, 5)
        dt = _timed_ranks(step, steps, 3, dev, world)
        status = batch_status(ex, None, "config 5") if P else {"extractor": 0, "matcher": 0}
        tot = torch.tensor([float(ns.sum()) if P else 0.0, float(P)], dtype=torch.float64, device=dev)
        if world > 1:
            torch.distributed.all_reduce(tot)
        total_pairs = nb * PB
        assert int(tot[1]) == total_pairs, "every pair of every batch processed exactly once"
        # per-pair digest of mvuRight / mvDepth over the left keypoints, gathered in pair order, so
        # a sharded run can be compared with one rank array for array (tests/test_bench_ranks.py)
        local = {}
        if P:
            ur_h, dep_h, cnt_h = ur.cpu().numpy(), dep.cpu().numpy(), cnt.cpu().numpy()
            for j, t in enumerate(pairs):
                n = min(int(cnt_h[2 * j]), cap)
                local[t] = hashlib.sha256(ur_h[j, :n].tobytes() + dep_h[j, :n].tobytes()).hexdigest()
        if world > 1:
            parts = [None] * world
            torch.distributed.all_gather_object(parts, local)
            for d in parts:
                local.update(d)
        digest = hashlib.sha256("".join(local[t] for t in sorted(local)).encode()).hexdigest()[:16]
        out[tag] = {"stereo_frames_per_s": round(total_pairs * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 4),
                    "batches_per_step": nb, "pairs_per_rank": P,
                    "stereo_matches_per_pair": round(float(tot[0]) / total_pairs, 1),
                    "uright_depth_sha16": digest, "status": status}
        del ex, o
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_stereo(cv, W, H, NF, EUROC_MBF, 8)
    return out


def config5_shard(amd, dev, cv, pairs, W=752, H=480, NF=1200, mbf=EUROC_MBF):
    """One rank's share of config 5: the stereo pairs `pairs` (indices into the synthetic EuRoC
    stream of canvas `cv`) resident in HBM as frames (2j, 2j+1) = (left, right) of one batch.  The
    returned step() runs orb_extract_batch_device over all 2P images (the two extractor roles of
    R/src/Frame.cpp:86-89 in one launch) and orb_compute_stereo_matches_batch_device
    (Frame::ComputeStereoMatches, R/src/Frame.cpp:551-770) on the device pyramids, on the current
    stream.  Returns (step, buffers); tests/test_bench_pipeline.py runs it against the oracle."""
    from orb_slam2_amd import synth, _abi
    lib = _abi.lib()
    P = len(pairs)
    ex = amd.ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index or 0, max_w=W, max_h=H, max_batch=max(2 * P, 1))
    cap = C.c_int()
    _abi.check("geom", lib.orb_extractor_geometry(ex._h, W, H, None, None, None, C.byref(cap)))
    cap = cap.value
    st = torch.cuda.current_stream(dev).cuda_stream
    o = {"ex": ex, "cap": cap, "P": P, "ur": None, "dep": None, "ns": None, "cnt": None, "frames": None}
    if P == 0:      # more ranks than pairs: this rank idles in the timed region
        return (lambda: None), o
    fr = np.stack([im for t in pairs for im in synth.stereo_pair(cv, W, H, t)])
    imgs = torch.from_numpy(fr).to(dev)
    kps = torch.zeros((2 * P, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((2 * P, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(2 * P, dtype=torch.int32, device=dev)
    ur = torch.zeros((P, cap), dtype=torch.float32, device=dev)
    dep = torch.zeros_like(ur)
    ns = torch.zeros(P, dtype=torch.int32, device=dev)
    o.update(frames=fr, imgs=imgs, kps=kps, desc=desc, cnt=cnt, ur=ur, dep=dep, ns=ns)

    def step():
        _abi.check("x", lib.orb_extract_batch_device(ex._h, C.c_void_p(imgs.data_ptr()), H * W, 2 * P, W, H,
                                                      C.c_void_p(kps.data_ptr()), C.c_void_p(desc.data_ptr()),
                                                      cap, C.c_void_p(cnt.data_ptr()), C.c_void_p(st)))
        _abi.check("stereo", lib.orb_compute_stereo_matches_batch_device(
            ex._h, C.c_void_p(kps.data_ptr()), C.c_void_p(desc.data_ptr()), C.c_void_p(cnt.data_ptr()), cap, P,
            C.c_float(mbf), C.c_float(0.0), C.c_void_p(ur.data_ptr()), C.c_void_p(dep.data_ptr()),
            C.c_void_p(ns.data_ptr()), C.c_void_p(st)))
    return step, o


def cpu_baseline_stereo(cv, W, H, NF, mbf, n_pairs):
    """Oracle: both images of each pair extracted (1 pair per host thread) + ComputeStereoMatches."""
    from orb_slam2_amd import synth
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ref as O
    p = O.params(NF)
    threads = host_threads()
    prs = [synth.stereo_pair(cv, W, H, t) for t in range(n_pairs)]

    def one(lr):
        a = O.extract(p, lr[0], want_pyramid=True)
        b = O.extract(p, lr[1], want_pyramid=True)
        return O.compute_stereo_matches(p, a, b, mbf)[0]
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as pool:
        list(pool.map(one, prs))
    dt = time.perf_counter() - t0
    return {"stereo_frames_per_s": round(n_pairs / dt, 2), "cores": threads, "kind": "port",
            "cpu_model": host_info()["cpu_model"],
            "sample": f"{n_pairs} stereo pairs {W}x{H}, {NF} feat: both images extracted + ComputeStereoMatches, "
                      f"oracle C restatement, 1 pair per host thread"}


KITTI_MBF = float(np.float32(_camera("KITTI00")["bf"]))   # R/Examples/Stereo/KITTI00-02.yaml Camera.bf


def bench_stereo_kitti(args, amd, dev, P=32):
    """BASELINE config 3, stereo: KITTI 00 geometry 1241x376, 2000 feat; per pair both images
    extracted + Frame::ComputeStereoMatches with the KITTI bf, HBM-resident, one GPU."""
    from orb_slam2_amd import synth, _abi
    lib = _abi.lib()
    W, H, NF = 1241, 376, 2000
    cv = synth.canvas(0x5EED0003, W, H)
    fr = np.stack([im for t in range(P) for im in synth.stereo_pair(cv, W, H, t)])
    ns = torch.zeros(P, dtype=torch.int32, device=dev)
    o = {}

    def stereo(b):
        if "ur" not in o:     # [P][cap] outputs at the extractor's keypoint capacity stride
            o["ur"] = torch.zeros((P, b["cap"]), dtype=torch.float32, device=dev)
            o["dep"] = torch.zeros_like(o["ur"])
        _abi.check("stereo", lib.orb_compute_stereo_matches_batch_device(
            b["ex"]._h, C.c_void_p(b["kps"].data_ptr()), C.c_void_p(b["desc"].data_ptr()),
            C.c_void_p(b["cnt"].data_ptr()), b["cap"], P, C.c_float(KITTI_MBF), C.c_float(0.0),
            C.c_void_p(o["ur"].data_ptr()), C.c_void_p(o["dep"].data_ptr()), C.c_void_p(ns.data_ptr()),
            C.c_void_p(b["stream"])))
    dt, b = _extract_leg(amd, dev, fr, NF, 10, 3, stereo)
    out = {"stereo_frames_per_s": round(P / dt, 1), "ms_per_step": round(dt * 1e3, 4), "pairs_per_step": P,
           "keypoints_per_image": float(b["cnt"].float().mean()),
           "stereo_matches_per_pair": float(ns.float().mean()), "status": b["status"],
           "config": f"synthetic KITTI 00 geometry {W}x{H} stereo (smooth integer disparity 5..60 px), {NF} feat, "
                     f"mbf {KITTI_MBF}, mb 0 (reference call order)"}
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_stereo(cv, W, H, NF, KITTI_MBF, 8)
    return out


def kitti_sfi_leg(amd, dev, m, B=64, steps=10, warmup=3):
    """BASELINE config 3 (KITTI 00 geometry 1241x376, 2000 feat, 8 levels): one step = B
    HBM-resident synthetic frames through orb_extract_batch_device, then
    orb_search_for_initialization_batch_device on the B-1 in-batch pairs (t-1, t) with window 100
    (R/src/ORBmatcher.cpp:499-617, as R/src/Tracking.cpp:779-780 calls it).  Returns (seconds per
    step, buffers incl. m12 / nm and both handles' status, the host frames);
    tests/test_bench_pipeline.py runs this same leg against the oracle."""
    from orb_slam2_amd import synth, _abi
    lib = _abi.lib()
    W, H = 1241, 376
    cv = synth.canvas(0x5EED0003, W, H)
    fr = np.stack([synth.frame(cv, W, H, t) for t in range(B)])
    o = {}

    def sfi(b):
        cp = b["cap"]
        if "m12" not in o:
            o["m12"] = torch.zeros((B - 1, cp), dtype=torch.int32, device=dev)
            o["nm"] = torch.zeros(B - 1, dtype=torch.int32, device=dev)
        _abi.check("sfi", lib.orb_search_for_initialization_batch_device(
            m._h, C.c_void_p(b["kps"].data_ptr()), C.c_void_p(b["desc"].data_ptr()), C.c_void_p(b["cnt"].data_ptr()),
            C.c_void_p(b["kps"].data_ptr() + cp * 28), C.c_void_p(b["desc"].data_ptr() + cp * 32),
            C.c_void_p(b["cnt"].data_ptr() + 4), B - 1, cp, W, H, 100, C.c_void_p(o["m12"].data_ptr()),
            C.c_void_p(o["nm"].data_ptr()), C.c_void_p(b["stream"])))
    dt, b = _extract_leg(amd, dev, fr, 2000, steps, warmup, sfi, matcher=m)
    b.update(o)
    return dt, b, fr


def bench_extras(args, amd, dev):
    """Secondary legs of SURVEY §8d: (ii) all-pairs 2-NN Hamming throughput (integer-VALU
    roofline: 16 lane-ops per 256-bit pair), config 5 stereo (EuRoC 752x480, 1200 feat,
    extraction of both images + ComputeStereoMatches), config 3 (KITTI 1241x376, 2000 feat,
    extract + SearchForInitialization)."""
    from orb_slam2_amd import synth, _abi
    lib = _abi.lib()
    out = {}
    # ---- (ii) brute-force 2-NN between consecutive frames' descriptors (1000 x 1000 per pair)
    W, H, B = 640, 480, 64
    cv = synth.canvas(0x5EED0002, W, H)
    frames = np.stack([synth.frame(cv, W, H, t) for t in range(B + 1)])
    _, buf = _extract_leg(amd, dev, frames, 1000, 1, 1)
    m = amd.ORBmatcher(0.9, True, device=dev.index or 0)
    cap = buf["cap"]
    nq = buf["cnt"][:-1].clone()
    bi = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    bd = torch.zeros_like(bi)
    sd = torch.zeros_like(bi)
    d = buf["desc"]
    st = buf["stream"]

    def knn():
        _abi.check("knn", lib.orb_hamming_knn2_batch_device(
            m._h, C.c_void_p(d.data_ptr()), C.c_void_p(nq.data_ptr()), C.c_void_p(d.data_ptr() + cap * 32),
            C.c_void_p(buf["cnt"].data_ptr() + 4), B, cap, cap, C.c_void_p(bi.data_ptr()), C.c_void_p(bd.data_ptr()),
            C.c_void_p(sd.data_ptr()), C.c_void_p(st)))
    for _ in range(3):
        knn()
    torch.cuda.synchronize(dev)
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        knn()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    c = buf["cnt"].cpu().numpy().astype(np.int64)
    pairs = float((c[:-1] * c[1:]).sum())
    # 16 lane-ops per pair (8 xor + 8 bcnt on dword pairs); 78.6 T lane-ops/s nominal (4 SIMD x 32
    # lanes per CU per clock), 41.7 T measured for integer VOP3 issue (profiles/r05_valu_issue.txt)
    peak_pairs = VALU_PEAK_TOPS * 1e12 / 16
    out["knn2_bruteforce"] = {"pairs_per_s": round(pairs / dt, 1), "ms_per_batch": round(dt * 1e3, 4),
                              "frame_pairs": B, "roofline": {"bound": "valu", "unit": "pairs/s",
                                                             "peak": peak_pairs, "frac": round(pairs / dt / peak_pairs, 4),
                                                             "frac_of_measured_issue_peak":
                                                                 round(pairs / dt / (VALU_MEASURED_TOPS * 1e12 / 16), 4)}}
    # ---- config 3 stereo: KITTI 00 geometry pairs, extraction of both images + ComputeStereoMatches
    out["stereo_kitti_1241x376"] = bench_stereo_kitti(args, amd, dev)
    # ---- config 3: KITTI geometry, 2000 features, extract + SearchForInitialization
    B = 64
    dt, b, _ = kitti_sfi_leg(amd, dev, m, B, 10, 3)
    out["kitti_1241x376"] = {"frames_per_s": round(B / dt, 1), "ms_per_step": round(dt * 1e3, 4),
                             "keypoints_per_frame": float(b["cnt"].float().mean()),
                             "matches_per_pair": float(b["nm"].float().mean()), "status": b["status"]}
    out["batch_sweep_640x480"] = batch_sweep(amd, dev, m)
    out["pose_optimization"] = bench_pose(args, amd, dev)
    out["single_call_latency"] = bench_single_calls(args, amd, dev)
    out["bow_transform"] = bench_bow(args, amd, dev)
    out["global_ba"] = bench_gba(args, amd, dev)
    return out


def bench_single_calls(args, amd, dev, reps=50):
    """The host-buffer entry points the C++ shims call once per frame / keyframe, timed one call
    at a time (median of `reps`, after warm-up; PCIe both ways included): ORBextractor::operator()
    on one 640x480 image (orb_extract: image in, keypoints + descriptors out), SearchForInitialization
    on one pair of those frames (orb_search_for_initialization), PoseOptimization of one frame
    (pose_optimize_batch, B = 1: frame in, pose + outlier flags out).  lba_solve's host path is
    the `lba` leg."""
    from orb_slam2_amd import synth, _abi, optimizer as opt
    import ctypes as C

    def med(fn):
        for _ in range(5):
            fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return round(1e6 * float(np.median(ts)), 1)
    cv = synth.canvas(0x5EED0002, 640, 480)
    img0, img1 = (np.ascontiguousarray(synth.frame(cv, 640, 480, t)) for t in (0, 1))
    ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, device=dev.index or 0)
    out = {"orb_extract_640x480_us": med(lambda: ex(img0))}
    k0, d0 = ex(img0)
    k1, d1 = ex(img1)
    m = amd.ORBmatcher(0.9, True, device=dev.index or 0)
    f0, f1 = amd.Frame(k0, d0, 640, 480), amd.Frame(k1, d1, 640, 480)
    prev = np.stack([k0["x"], k0["y"]], 1).astype(np.float32)
    out["search_for_initialization_us"] = med(lambda: m.SearchForInitialization(f0, f1, prev.copy(), 100))
    fr = synth.pose_problems(n_frames=1, n_points=600, stereo_frac=0.3, seed=21)
    a = opt.pack_pose_frames(fr)
    E = int(a["edge_start"][-1])
    pb = opt.PoseBatch(1, E, _abi.ptr(a["pose_q"]), _abi.ptr(a["pose_t"]), _abi.ptr(a["cam"]), _abi.ptr(a["edge_start"]),
                       _abi.ptr(a["edge_obs"]), _abi.ptr(a["edge_xw"]), _abi.ptr(a["edge_info"]))
    q, t = np.zeros((1, 4)), np.zeros((1, 3))
    outl, ninl, iters = np.zeros(E, np.uint8), np.zeros(1, np.int32), np.zeros((1, 5), np.int32)
    r = opt.PoseBatchResult(_abi.ptr(q), _abi.ptr(t), _abi.ptr(outl), _abi.ptr(ninl))
    lib, devi = opt._pose_sig(), dev.index or 0
    out["pose_optimization_one_frame_us"] = med(
        lambda: _abi.check("pose", lib.pose_optimize_batch(devi, C.byref(pb), C.byref(r), _abi.ptr(iters))))
    out["note"] = ("host buffers, PCIe both ways, one call at a time (median); each call is a chain of dependent "
                   "launches + copies, so these are launch/transfer latencies, not throughput")
    out["routed_calls"] = bench_routed_calls(args, amd, dev, med)
    return out


def bench_routed_calls(args, amd, dev, med, creps=9):
    """Every other matcher / optimizer call the drop-in routes to the library, one call at
    a time through its host-buffer entry point at the reference's call size (~1000 keypoints per
    keyframe, TUM), against the oracle's restatement of the same call on one host thread (median of
    `creps`; the reference runs these single-threaded on the LocalMapping / Tracking / LoopClosing
    threads).  Each row: gpu_us, cpu_1thread_us, the reference call site.  LocalBundleAdjustment is
    timed through the compiled C++ shim (graph gather R/src/Optimizer.cpp:569-625 + solve +
    write-back :883-917, orb-slam2-_amd/lib/shim_caller timeit) on the config-4 window."""
    from orb_slam2_amd import synth, Frame
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ref as O
    rows = {}

    def cmed(fn):
        fn()
        ts = []
        for _ in range(creps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return round(1e6 * float(np.median(ts)), 1)

    def row(name, gpu_fn, cpu_fn, site, size):
        g = med(gpu_fn)
        c = None if args.no_cpu else cmed(cpu_fn)
        rows[name] = {"gpu_us": g, "cpu_1thread_us": c, "gpu_over_cpu": None if c is None else round(c / g, 2),
                      "call_site": site, "size": size}

    def kp_of(k, angle=True):
        a = np.zeros(len(k["x"]), dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                         ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
        a["x"], a["y"], a["octave"] = k["x"], k["y"], k["octave"]
        if angle and "angle" in k:
            a["angle"] = k["angle"]
        return a
    # SearchByBoW(KF, Frame) and (KF, KF)
    voc = synth.vocabulary(k=10, L=4, seed=5, early_leaf=0.05, stop_frac=0.03)
    ov = O.OracleVocabulary(*voc, 4)
    k1, k2 = synth.bow_match_problem(voc, seed=11)
    # FeatureVector at level L - levelsup = 2 (this 4-level vocabulary, levelsup 2): the node granularity of
    # the reference's ORBvoc (L = 6) with its levelsup 4 (R/src/Frame.cpp:465, R/src/KeyFrame.cpp:72), ~100
    # nodes of ~10 features per side.  (levelsup 4 here would put every feature in the root node: one
    # 900 x 900 node, one workgroup — not a call the reference makes.)
    fv1, fv2 = O.bow_transform(ov, k1["desc"], 2)[1], O.bow_transform(ov, k2["desc"], 2)[1]
    a1, a2 = O.featvec_arrays(fv1), O.featvec_arrays(fv2)
    f1, f2 = Frame(kp_of(k1), k1["desc"], k1["W"], k1["H"]), Frame(kp_of(k2), k2["desc"], k2["W"], k2["H"])
    m = amd.ORBmatcher(0.7, True, device=dev.index or 0)
    size = f"{len(k1['x'])} x {len(k2['x'])} features, {len(fv1)} / {len(fv2)} level-2 nodes"
    row("search_by_bow_kf_frame", lambda: m.SearchByBoW(f1, k1["has_mp"], a1, f2, a2),
        lambda: O.search_by_bow_frame(k1, k1["has_mp"], a1, k2, a2, 0.7, True), "R/src/Tracking.cpp:1020, 1840", size)
    row("search_by_bow_kf_kf", lambda: m.SearchByBoWKF(f1, k1["has_mp"], a1, f2, k2["has_mp"], a2),
        lambda: O.search_by_bow_kf(k1, k1["has_mp"], a1, k2, k2["has_mp"], a2, 0.7, True), "R/src/LoopClosing.cpp:327", size)
    # SearchForTriangulation
    tp = synth.triangulation_problem()
    t1, t2 = tp["kf1"], tp["kf2"]
    tf1 = Frame(kp_of(t1), t1["desc"], t1["W"], t1["H"], mvuRight=t1["uright"])
    tf2 = Frame(kp_of(t2), t2["desc"], t2["W"], t2["H"], mvuRight=t2["uright"])
    row("search_for_triangulation",
        lambda: amd.SearchForTriangulation(tf1, tf2, t1["has_mp"], t2["has_mp"], (t1["nodes"], t1["start"], t1["fidx"]),
                                           (t2["nodes"], t2["start"], t2["fidx"]), tp["F12"], (tp["ex"], tp["ey"]),
                                           tp["scale_factors"], tp["level_sigma2"], False, True),
        lambda: O.search_for_triangulation(tp, False, True), "R/src/LocalMapping.cpp:374",
        f"{len(t1['x'])} x {len(t2['x'])} keypoints")
    # Fuse (keyframe, map points) and the Scw form; SearchByProjection(KF, Scw)
    fp = synth.fuse_problem()
    kf, kp = fp["kf"], fp["kp"]
    ff = Frame(kp_of(kf, False), kf["desc"], kf["W"], kf["H"], mvuRight=kf["uright"])
    fargs = (fp["mp_valid"], fp["mp_xyz"], fp["mp_normal"], fp["mp_min_dist"], fp["mp_max_dist"], fp["mp_desc"])
    fsize = f"{len(kf['x'])} keypoints, {len(fp['mp_xyz'])} map points"
    row("fuse", lambda: amd.Fuse(ff, kp["Tcw"], kp["Ow"], kp["cam"], kp["log_scale_factor"], kp["scale_factors"],
                                 kp["inv_level_sigma2"], *fargs, 3.0),
        lambda: O.fuse(fp, 3.0), "R/src/LocalMapping.cpp:654, 688", fsize)
    pre = np.full(len(kf["x"]), -1, np.int32)
    row("search_by_projection_sim3",
        lambda: m.SearchByProjectionSim3(ff, np.asarray(kp["Tcw"], np.float32)[:3, :4], kp["Ow"], kp["cam"],
                                         kp["log_scale_factor"], kp["scale_factors"], *fargs, 10.0, pre.copy()),
        lambda: O.search_by_projection_sim3(fp, 10.0, pre.copy()), "R/src/LoopClosing.cpp:474", fsize)
    # SearchByProjection(Frame, KF, set, th, ORBdist) (relocalisation)
    rng = np.random.default_rng(103)
    n_mp = len(fp["mp_xyz"])
    kfs = {"x": rng.uniform(0, 640, n_mp).astype(np.float32), "y": rng.uniform(0, 480, n_mp).astype(np.float32),
           "octave": np.zeros(n_mp, np.int32), "desc": np.zeros((n_mp, 32), np.uint8),
           "angle": rng.uniform(0, 360, n_mp).astype(np.float32), "W": 640, "H": 480}
    kfa = dict(kf, angle=rng.uniform(0, 360, len(kf["x"])).astype(np.float32))
    T = np.eye(4, dtype=np.float32)
    T[:3, :4] = np.asarray(kp["Tcw"], np.float32)[:3, :4]
    fcur = Frame(kp_of(kfa), kfa["desc"], kfa["W"], kfa["H"], mTcw=T, mvScaleFactors=np.asarray(kp["scale_factors"], np.float32))
    fks = Frame(kp_of(kfs), kfs["desc"], 640, 480)
    occ = np.full(len(kf["x"]), -1, np.int32)
    cur_v, kf_v = O.FrameView(kfa, kfa["desc"], 640, 480), O.FrameView(kfs, kfs["desc"], 640, 480)
    row("search_by_projection_kf",
        lambda: m.SearchByProjectionKF(fcur, fks, fp["mp_valid"], fp["mp_xyz"], fp["mp_min_dist"], fp["mp_max_dist"],
                                       fp["mp_desc"], kp["cam"][:4], kp["Ow"], kp["log_scale_factor"], 10.0, 100, occ.copy()),
        lambda: O.search_by_projection_kf(cur_v, kp["Tcw"][:3, :4], kp["Ow"], kf_v, fp["mp_valid"], fp["mp_xyz"],
                                          fp["mp_min_dist"], fp["mp_max_dist"], fp["mp_desc"], kp["cam"][:4],
                                          kp["log_scale_factor"], kp["scale_factors"], 10.0, 100, True, occ.copy()),
        "R/src/Tracking.cpp:1921", fsize)
    # SearchBySim3
    sp = synth.sim3_problem()
    S1, S2 = synth.sim3_side_transforms(sp)
    sides = [dict(Tcw=k["Tcw"], S=S, valid=k["mp_valid"], xyz=k["mp_xyz"], min_dist=k["mp_min_dist"],
                  max_dist=k["mp_max_dist"], desc=k["mp_desc"]) for k, S in ((sp["kf1"], S1), (sp["kf2"], S2))]
    sc = (sp["log_scale_factor"], sp["scale_factors"])
    sf1 = Frame(kp_of(sp["kf1"], False), sp["kf1"]["desc"], 640, 480)
    sf2 = Frame(kp_of(sp["kf2"], False), sp["kf2"]["desc"], 640, 480)
    row("search_by_sim3", lambda: amd.SearchBySim3(sf1, sf2, sides[0], sides[1], sp["cam"], sc, sc, 7.5),
        lambda: O.search_by_sim3(sp, 7.5), "R/src/LoopClosing.cpp:402",
        f"{len(sp['kf1']['x'])} x {len(sp['kf2']['x'])} keypoints")
    # ComputeDistinctiveDescriptors (per new map point: its observations' descriptors)
    drng = np.random.default_rng(5)
    lists = [drng.integers(0, 256, (int(drng.integers(2, 9)), 32), dtype=np.uint8) for _ in range(300)]
    row("compute_distinctive_descriptors_300_points", lambda: amd.ComputeDistinctiveDescriptors(lists, device=dev.index or 0),
        lambda: [O.distinctive_descriptor(l) for l in lists], "R/src/LocalMapping.cpp:467 (one call per point)",
        "300 map points x 2-8 observations")
    # Frame::ComputeStereoMatches (EuRoC geometry) after the two extractions
    W, H, NF = 752, 480, 1200
    left, right = synth.stereo_pair(synth.canvas(0x5EED0005, W, H), W, H, 0)
    exL = amd.ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index or 0, max_w=W, max_h=H)
    exR = amd.ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index or 0, max_w=W, max_h=H)
    kl, dl = exL(left)
    kr, dr = exR(right)
    pp = O.params(NF)
    ea, eb = O.extract(pp, left, want_pyramid=True), O.extract(pp, right, want_pyramid=True)
    row("compute_stereo_matches_euroc", lambda: amd.ComputeStereoMatches(exL, exR, kl, dl, kr, dr, EUROC_MBF),
        lambda: O.compute_stereo_matches(pp, ea, eb, EUROC_MBF), "R/src/Frame.cpp:101",
        f"{len(kl)} x {len(kr)} keypoints, 752x480")
    m.close()
    # LocalBundleAdjustment through the compiled shim (config 4 window)
    exe = ROOT / "orb-slam2-_amd" / "lib" / "shim_caller"
    if exe.exists():
        import subprocess
        import tempfile
        pb = synth.ba_problem(n_local=args.lba_kf, n_points=args.lba_points)
        inv_sigma2 = (np.float32(1.0) / np.array([np.float32(1.2) ** (2 * lv) for lv in range(8)], np.float32))
        octave = np.array([int(np.argmin(np.abs(inv_sigma2.astype(np.float64) - i))) for i in pb["edge_info"]], np.int32)
        arrays = [np.asarray(pb["Tcw"], np.float32).reshape(-1), np.asarray(pb["pose_fixed"], np.uint8),
                  np.asarray(pb["pose_id"], np.int64), np.asarray(pb["point_xyz"], np.float32).reshape(-1),
                  np.asarray(pb["point_id"], np.int64), np.asarray(pb["edge_point"], np.int32),
                  np.asarray(pb["edge_pose"], np.int32), np.asarray(pb["edge_obs"], np.float32).reshape(-1), octave,
                  np.asarray(pb["edge_cam"][0], np.float32), inv_sigma2, np.zeros(1, np.uint8)]
        with tempfile.TemporaryDirectory() as td:
            inp = pathlib.Path(td) / "lba.in"
            with open(inp, "wb") as f:
                for a in arrays:
                    a = np.ascontiguousarray(a)
                    np.array([a.size], np.int64).tofile(f)
                    a.tofile(f)
            res = subprocess.run([str(exe), "timeit", "20", "lba", str(inp)], capture_output=True, text=True,
                                 timeout=300)
            resc = None
            if not args.no_cpu:   # the same shim gather / write-back around the oracle's 1-thread solve
                env = dict(os.environ, ORB_ORACLE_LIB=str(ROOT / "oracle" / "build" / "liborb_oracle.so"))
                resc = subprocess.run([str(exe), "timeit", "3", "lbacpu", str(inp)], capture_output=True, text=True,
                                      timeout=600, env=env)

        def parse(r):
            if r is None or r.returncode != 0 or not r.stdout.startswith("median_us"):
                return None, None
            w = r.stdout.split()
            ph = None
            if "phases_us" in w:
                i = w.index("phases_us")
                ph = dict(zip(("gather", "arrays", "lba_solve", "write_back"), (float(x) for x in w[i + 1:i + 5])))
            return float(w[1]), ph
        g, gph = parse(res)
        c, cph = parse(resc)
        rows["local_bundle_adjustment_shim"] = {
            "gpu_us": g, "cpu_1thread_us": c, "gpu_over_cpu": None if (c is None or not g) else round(c / g, 2),
            "gpu_phases_us": gph, "cpu_phases_us": cph,
            "host_pool_threads": int(os.environ.get("ORB_SHIM_THREADS", "4")),
            "call_site": "R/src/LocalMapping.cpp:95", "size": f"{args.lba_kf} KF + 4 fixed x {args.lba_points} points",
            "note": "whole call through the compiled drop-in: window gather from the (mock) map, the problem arrays, "
                    "the solve, vToErase + write-back (phase medians); cpu = the same shim code around the oracle's "
                    "single-threaded solve (the reference's LocalMapping runs g2o without OpenMP)",
            "stderr_tail": None if res.returncode == 0 else res.stderr[-300:]}
    return rows


def bench_pose(args, amd, dev, n_frames=256, n_points=600):
    """Optimizer::PoseOptimization over a batch of synthetic frames (600 matched
    map points each, 10 % displaced, 30 % stereo), inputs resident in HBM, one workgroup per
    frame; against the oracle (C restatement of the reference, 1 thread per frame, 16 threads)."""
    from orb_slam2_amd import synth, _abi, optimizer as opt
    frames = synth.pose_problems(n_frames=n_frames, n_points=n_points, stereo_frac=0.3, seed=21)
    a = opt.pack_pose_frames(frames)
    B, E = n_frames, int(a["edge_start"][-1])
    T = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in a.items()}
    pq = torch.zeros((B, 4), dtype=torch.float64, device=dev)
    pt = torch.zeros((B, 3), dtype=torch.float64, device=dev)
    outl = torch.zeros(E, dtype=torch.uint8, device=dev)
    ninl = torch.zeros(B, dtype=torch.int32, device=dev)
    work = torch.zeros(3 * E, dtype=torch.float64, device=dev)
    flags = torch.zeros(2 * E, dtype=torch.uint8, device=dev)
    iters = torch.zeros((B, 5), dtype=torch.int32, device=dev)
    dp = lambda x: C.c_void_p(x.data_ptr())   # noqa: E731
    pb = opt.PoseBatch(B, E, dp(T["pose_q"]), dp(T["pose_t"]), dp(T["cam"]), dp(T["edge_start"]), dp(T["edge_obs"]),
                       dp(T["edge_xw"]), dp(T["edge_info"]))
    pr = opt.PoseBatchResult(dp(pq), dp(pt), dp(outl), dp(ninl))
    lib = opt._pose_sig()
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run():
        _abi.check("pose", lib.pose_optimize_batch_device(C.byref(pb), C.byref(pr), dp(work), dp(flags), dp(iters),
                                                          C.c_void_p(stream)))
    for _ in range(2):
        run()
    torch.cuda.synchronize(dev)
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    it = iters.cpu().numpy()
    out = {"frames_per_s": round(B / dt, 1), "ms_per_batch": round(dt * 1e3, 4), "frames_per_batch": B,
           "edges_per_frame": n_points, "lm_iterations_per_frame": float(it[:, :4].sum(1).mean()),
           "trials_per_frame": float(it[:, 4].mean()),
           "inliers_per_frame": float(ninl.float().mean())}
    if not args.no_cpu:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_ref as O
        sample = frames[:64]
        threads = host_threads()
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            list(ex.map(O.pose_optimization, sample))
        dc = time.perf_counter() - t0
        out["cpu_baseline"] = {"frames_per_s": round(len(sample) / dc, 1), "cores": threads, "kind": "port",
                               "sample": f"{len(sample)} frames, oracle C restatement of PoseOptimization, "
                                         f"1 frame per thread"}
    return out


def bench_gba(args, amd, dev, n_kf=60, n_points=8000, iters=10):
    """Optimizer::BundleAdjustment (LoopClosing's 10 iterations, bRobust false) on a
    synthetic 60-keyframe, 8000-point map (reduced camera system 360 x 360): wall time of the
    whole call (host structure build, transfers, kernels); against the oracle on the same map."""
    from orb_slam2_amd import synth
    pb = synth.ba_problem(n_local=n_kf, n_fixed=0, n_points=n_points, seed=17, arc=6.0)
    ctx = amd.LocalBA()
    from orb_slam2_amd import optimizer as opt
    o = opt.global_options(iters)
    ctx.solve(pb, o, global_ba=True, robust=False)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        r = ctx.solve(pb, o, global_ba=True, robust=False)
    dt = (time.perf_counter() - t0) / reps
    it = r["iterations"][0]
    out = {"ms_per_call": round(dt * 1e3, 3), "ms_per_iteration": round(dt * 1e3 / max(it, 1), 3),
           "iterations": it, "keyframes": n_kf, "points": n_points, "edges": int(len(pb["edge_point"]))}
    if not args.no_cpu:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_ref as O
        t0 = time.perf_counter()
        ref = O.global_ba(pb, iters, robust=False)
        dc = time.perf_counter() - t0
        out["cpu_baseline"] = {"ms_per_call": round(dc * 1e3, 2), "cores": 1, "kind": "port",
                               "sample": "the same map, oracle C restatement of g2o LM + Schur, 1 thread",
                               "same_iterations": ref["iterations"][0] == it}
    ctx.close()
    return out


def bench_bow(args, amd, dev, n_frames=64, n_feat=1000):
    """DBoW2 TemplatedVocabulary::transform (ComputeBoW, levelsup 4) for a batch of
    frames' descriptors resident in HBM against a synthetic vocabulary of the ORBvoc.txt shape
    (k=10, L=6, 10^6 words, 35.6 MB of node descriptors); against the oracle C restatement."""
    from orb_slam2_amd import synth, _abi
    parent, leaf, desc, weight = synth.vocabulary(k=10, L=6, seed=7, early_leaf=0.0, dup_frac=0.0)
    voc = amd.ORBVocabulary.from_nodes(parent, leaf, desc, weight, k=10, L=6)
    n = n_frames * n_feat
    feats = synth.bow_features(desc, leaf, n, seed=13)
    d_f = torch.from_numpy(feats).to(dev)
    d_w = torch.zeros(n, dtype=torch.int32, device=dev)
    d_g = torch.zeros(n, dtype=torch.float64, device=dev)
    d_n = torch.zeros(n, dtype=torch.int32, device=dev)
    lib = _abi.lib()
    lib.orb_vocabulary_transform_device.argtypes = [C.c_void_p] * 2 + [C.c_int, C.c_int] + [C.c_void_p] * 4
    lib.orb_vocabulary_transform_device.restype = C.c_int
    h = voc._handle()
    stream = torch.cuda.current_stream(dev).cuda_stream
    dp = lambda x: C.c_void_p(x.data_ptr())   # noqa: E731

    def run():
        _abi.check("bow", lib.orb_vocabulary_transform_device(h, dp(d_f), n, 4, dp(d_w), dp(d_g), dp(d_n),
                                                              C.c_void_p(stream)))
    for _ in range(3):
        run()
    torch.cuda.synchronize(dev)
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize(dev)
    dt = e0.elapsed_time(e1) / 1e3 / reps
    # bytes a descriptor touches: its 32 B in, per level one 8 B (first child, count) record and 10
    # adjacent 32 B child descriptors, 4 + 8 + 4 B word / weight / node id out plus the 4 B node map
    per = 32 + 6 * (8 + 10 * 32) + 20
    out = {"descriptors_per_s": round(n / dt, 1), "frames_per_s": round(n_frames / dt, 1),
           "ms_per_batch": round(dt * 1e3, 4), "frames_per_batch": n_frames, "descriptors_per_frame": n_feat,
           "vocabulary": "k=10 L=6, 1111111 nodes, 10^6 words (synthetic, ORBvoc.txt shape)",
           "touched_GBps": round(n * per / dt / 1e9, 1), "touched_bytes_per_descriptor": per}
    if not args.no_cpu:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_ref as O
        ov = O.OracleVocabulary(parent, leaf, desc, weight, 6)
        m = 20000
        t0 = time.perf_counter()
        rw, _, _ = O.vocab_transform(ov, feats[:m], 4)
        dc = time.perf_counter() - t0
        ok = bool(np.array_equal(rw, d_w[:m].cpu().numpy()))
        out["cpu_baseline"] = {"descriptors_per_s": round(m / dc, 1), "cores": 1, "kind": "port",
                               "sample": f"{m} descriptors, oracle C restatement of transform, 1 thread",
                               "word_ids_match": ok}
    del voc
    return out


def batch_sweep(amd, dev, m):
    """extract + SearchForInitialization at batch sizes B in {1, 8, 64} on one stream,
    HBM-resident (B-1 in-batch pairs; B=1 is extraction alone), and the PCIe-inclusive rate at the
    same sizes: pinned host frames copied in, keypoints + descriptors + matches copied back, per step."""
    from orb_slam2_amd import synth, _abi
    lib = _abi.lib()
    W, H, NF = 640, 480, 1000
    cv = synth.canvas(0x5EED0002, W, H)
    res = {}
    for B in (1, 8, 64):
        fr = np.stack([synth.frame(cv, W, H, t) for t in range(B)])
        m12 = torch.zeros((max(B - 1, 1), 4096), dtype=torch.int32, device=dev)
        nm = torch.zeros(max(B - 1, 1), dtype=torch.int32, device=dev)

        def sfi(b, B=B, m12=m12, nm=nm):
            if B < 2:
                return
            cp = b["cap"]
            _abi.check("sfi", lib.orb_search_for_initialization_batch_device(
                m._h, C.c_void_p(b["kps"].data_ptr()), C.c_void_p(b["desc"].data_ptr()),
                C.c_void_p(b["cnt"].data_ptr()), C.c_void_p(b["kps"].data_ptr() + cp * 28),
                C.c_void_p(b["desc"].data_ptr() + cp * 32), C.c_void_p(b["cnt"].data_ptr() + 4), B - 1, cp, W, H,
                100, C.c_void_p(m12.data_ptr()), C.c_void_p(nm.data_ptr()), C.c_void_p(b["stream"])))
        dt, b = _extract_leg(amd, dev, fr, NF, 20 if B < 64 else 10, 3, sfi, matcher=m if B > 1 else None)
        res[f"B{B}"] = {"frames_per_s": round(B / dt, 1), "ms_per_step": round(dt * 1e3, 4), "status": b["status"]}
    # PCIe-inclusive, B = 1 / 8 / 64: H2D of the frames, extraction + matching, D2H of the results
    for B in (1, 8, 64):
        res[f"B{B}_pcie_inclusive"] = _pcie_leg(amd, dev, m, cv, W, H, NF, B)
    h2d, d2h = measure_pinned_copy(dev)
    res["pinned_copy_gbs"] = {"h2d": h2d, "d2h": d2h, "source": "64 MiB pinned host <-> device copies x10 on one "
                                                                "stream, HIP events, in this run"}
    for B in (8, 64):
        r = _pcie_pipelined_leg(amd, dev, cv, W, H, NF, B)
        r["h2d_bound_frames_per_s"] = round(h2d * 1e9 / r["h2d_bytes_per_step"] * B, 1)
        r["frac_of_h2d_bound"] = round(r["frames_per_s"] / r["h2d_bound_frames_per_s"], 3)
        # the same pipeline with its uploads alone (no compute, no compaction): the rate the copy
        # stream sustains for this batch's frames, the bound the whole leg meets (bench._pcie_pipelined_leg)
        old_part = os.environ.get("ORB_BENCH_PCIE_PART")
        os.environ["ORB_BENCH_PCIE_PART"] = "copy"
        try:
            up = _pcie_pipelined_leg(amd, dev, cv, W, H, NF, B)
        finally:
            if old_part is None:
                os.environ.pop("ORB_BENCH_PCIE_PART", None)
            else:
                os.environ["ORB_BENCH_PCIE_PART"] = old_part
        r["uploads_only_frames_per_s"] = up["frames_per_s"]
        r["frac_of_uploads_only"] = round(r["frames_per_s"] / up["frames_per_s"], 3)
        res[f"B{B}_pcie_pipelined"] = r
    return res


def measure_pinned_copy(dev, mib=64, reps=10):
    """Pinned host <-> device copy rates on one stream (HIP events around `reps` copies of `mib`
    MiB each way): the PCIe ceiling the PCIe-inclusive legs are read against."""
    n = mib << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    d.copy_(h, non_blocking=True)
    h.copy_(d, non_blocking=True)
    torch.cuda.synchronize(dev)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    for _ in range(reps):
        d.copy_(h, non_blocking=True)
    e[1].record()
    for _ in range(reps):
        h.copy_(d, non_blocking=True)
    e[2].record()
    torch.cuda.synchronize(dev)
    h2d = n * reps / (e[0].elapsed_time(e[1]) * 1e-3) / 1e9
    d2h = n * reps / (e[1].elapsed_time(e[2]) * 1e-3) / 1e9
    return round(h2d, 2), round(d2h, 2)


def _pcie_pipelined_leg(amd, dev, cv, W, H, NF, B, steps=48, warmup=4, check=None):
    """The PCIe-inclusive path as a streaming host would run it, on three HIP streams: the copy
    stream uploads batch s+1's pinned frames (one H2D, into one of three device frame buffers)
    while two compute streams, one per batch parity with its own extractor and matcher handles,
    run batches s and s-1: extraction, SearchForInitialization over the B-1 in-batch pairs, and
    the compaction of keypoints / descriptors / matches12 (orb_pack_rows_device), which stores
    exactly the counted rows straight into host-mapped pinned memory (no D2H copy command, no
    host wait for the counts).  Events order the hand-offs: a frame buffer is refilled only after
    the extraction that reads it in place (level 0, LEVEL-0 LIFETIME) has finished.  The host
    outputs rotate over three sets: before enqueueing batch s the host waits for batch s-3's
    outputs (a consumer reading them), so the GPU always holds the next batches' work.  The timed
    steps start from an idle pipeline and end with it drained (48 of them: the fill and the drain
    are ~1 batch each, ~4 % of the time); ORB_BENCH_PCIE_DEPTH sets the frame buffers / host output
    sets in flight (default 4: +0-3 % over 3 in same-box A/Bs).  What bounds it (tools/pcie_depth_ab.py,
    one box): the uploads alone run at 167-170 k frames/s, the compute alone at 211 k, uploads +
    compute without the compaction into host memory at 165-168 k (the overlap is complete: the
    upload stream binds), the whole leg at 150-160 k (the compaction's PCIe stores slow the
    uploads by 5-10 %)."""
    from orb_slam2_amd import synth, _abi
    lib = _abi.lib()
    hip = C.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipHostFree.argtypes = [C.c_void_p]
    hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]
    nb = 4   # distinct pinned host batches (inputs)
    host_in = [torch.from_numpy(np.stack([synth.frame(cv, W, H, t + k * B) for t in range(B)])).pin_memory()
               for k in range(nb)]
    exs = [amd.ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index or 0, max_w=W, max_h=H, max_batch=B) for _ in range(2)]
    ms = [amd.ORBmatcher(0.9, True, device=dev.index or 0) for _ in range(2)]
    cap = C.c_int()
    _abi.check("geom", lib.orb_extractor_geometry(exs[0]._h, W, H, None, None, None, C.byref(cap)))
    cap = cap.value
    P = max(B - 1, 1)
    s_copy, s_comps = torch.cuda.Stream(dev), [torch.cuda.Stream(dev) for _ in range(2)]
    depth = max(3, int(os.environ.get("ORB_BENCH_PCIE_DEPTH", "4")))
    NF_BUF = depth   # device frame buffers: the upload of batch s+1 never waits for batch s's extraction
    imgs = [torch.empty((B, H, W), dtype=torch.uint8, device=dev) for _ in range(NF_BUF)]
    ev_in = [torch.cuda.Event() for _ in range(NF_BUF)]     # frames of buffer f uploaded
    ev_ext = [torch.cuda.Event() for _ in range(NF_BUF)]    # extraction done reading buffer f
    kps = [torch.zeros((B, cap, 7), dtype=torch.int32, device=dev) for _ in range(2)]
    desc = [torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev) for _ in range(2)]
    cnt = [torch.zeros(B, dtype=torch.int32, device=dev) for _ in range(2)]
    m12 = [torch.zeros((P, cap), dtype=torch.int32, device=dev) for _ in range(2)]
    nm = [torch.zeros(P, dtype=torch.int32, device=dev) for _ in range(2)]
    sizes = {"pk": B * cap * 28, "pd": B * cap * 32, "pm": P * cap * 4, "off": 3 * (B + 1) * 4}
    NO = depth   # host output sets
    hostbufs, outs = [], []
    for _ in range(NO):   # host-mapped, coherent: the pack kernel's stores land in host memory
        o = {}
        for k, n in sizes.items():
            h, dptr = C.c_void_p(), C.c_void_p()
            if hip.hipHostMalloc(C.byref(h), n, 0x2 | 0x40000000) != 0 or \
                    hip.hipHostGetDevicePointer(C.byref(dptr), h, 0) != 0:
                raise SystemExit("pipelined PCIe leg: hipHostMalloc (mapped) failed")
            hostbufs.append(h)
            o[k] = (h, dptr)
        outs.append(o)
    dp = lambda x: C.c_void_p(x.data_ptr())   # noqa: E731
    moved = {"d2h": 0}
    ev_done = [torch.cuda.Event() for _ in range(NO)]   # host output set j written

    # diagnosis knobs (tools/pcie_depth_ab.py): ORB_BENCH_PCIE_PART=copy (uploads only), =compute (no
    # uploads: the frames stay resident), =nopack (no compaction into host memory); default: all
    part = os.environ.get("ORB_BENCH_PCIE_PART", "all")

    def enqueue(s):
        i, f = s % 2, s % NF_BUF
        o = outs[s % NO]
        if part == "copy":
            with torch.cuda.stream(s_copy):
                imgs[f].copy_(host_in[s % nb], non_blocking=True)
            ev_done[s % NO].record(s_copy)
            return
        if s >= NF_BUF:   # buffer f's previous extraction (batch s-3) must be done reading level 0
            s_copy.wait_event(ev_ext[f])
        if part != "compute":
            with torch.cuda.stream(s_copy):
                imgs[f].copy_(host_in[s % nb], non_blocking=True)
        ev_in[f].record(s_copy)
        s_comp = s_comps[i]   # batch s-2 ran on this stream before: set i is free in stream order
        s_comp.wait_event(ev_in[f])
        sp = C.c_void_p(s_comp.cuda_stream)
        k, d, c, mm = kps[i], desc[i], cnt[i], m12[i]
        _abi.check("x", lib.orb_extract_batch_device(exs[i]._h, dp(imgs[f]), H * W, B, W, H, dp(k), dp(d), cap, dp(c),
                                                      sp))
        ev_ext[f].record(s_comp)
        if B > 1:
            _abi.check("sfi", lib.orb_search_for_initialization_batch_device(
                ms[i]._h, dp(k), dp(d), dp(c), C.c_void_p(k.data_ptr() + cap * 28), C.c_void_p(d.data_ptr() + cap * 32),
                C.c_void_p(c.data_ptr() + 4), B - 1, cap, W, H, 100, dp(mm), dp(nm[i]), sp))
        off = o["off"][1].value
        if part == "nopack":
            ev_done[s % NO].record(s_comp)
            return
        _abi.check("pack", lib.orb_pack_rows_device(dp(k), 28, cap, dp(c), B, o["pk"][1], C.c_void_p(off), sp))
        _abi.check("pack", lib.orb_pack_rows_device(dp(d), 32, cap, dp(c), B, o["pd"][1], C.c_void_p(off + 4 * (B + 1)),
                                                    sp))
        if B > 1:   # vnMatches12 of pair (t-1, t) has frame t-1's N rows
            _abi.check("pack", lib.orb_pack_rows_device(dp(mm), 4, cap, dp(c), B - 1, o["pm"][1],
                                                        C.c_void_p(off + 8 * (B + 1)), sp))
        ev_done[s % NO].record(s_comp)

    def consume(s):   # the host reads batch s's outputs: totals from the mapped offsets
        ev_done[s % NO].synchronize()
        if part in ("copy", "nopack"):
            return
        o = outs[s % NO]
        offs = np.ctypeslib.as_array(C.cast(o["off"][0], C.POINTER(C.c_int32)), shape=(3, B + 1))
        n_kp, n_m = int(offs[0, B]), int(offs[2, B - 1]) if B > 1 else 0
        moved["d2h"] += n_kp * 60 + n_m * 4 + sizes["off"]
        if check is not None:   # (tests: the packed host outputs of batch s against the reference)
            view = lambda k, n, t: np.ctypeslib.as_array(C.cast(o[k][0], C.POINTER(t)), shape=(n,)).copy()  # noqa: E731
            check(s, host_in[s % nb].numpy(), offs.copy(), view("pk", n_kp * 7, C.c_int32).reshape(-1, 7),
                  view("pd", n_kp * 32, C.c_uint8).reshape(-1, 32), view("pm", max(n_m, 0), C.c_int32))

    def run(s0, n):
        for s in range(s0, s0 + n):
            if s - s0 >= NO:
                consume(s - NO)
            enqueue(s)
        for s in range(max(s0, s0 + n - NO), s0 + n):
            consume(s)
        torch.cuda.synchronize(dev)

    try:
        run(0, warmup)
        moved["d2h"] = 0
        t0 = time.perf_counter()
        run(warmup, steps)
        dt = (time.perf_counter() - t0) / steps
        st = [batch_status(e, mt, f"pipelined PCIe leg B={B}") for e, mt in zip(exs, ms)][0]
    finally:
        torch.cuda.synchronize(dev)
        for h in hostbufs:
            hip.hipHostFree(h)
    return {"frames_per_s": round(B / dt, 1), "ms_per_step": round(dt * 1e3, 4), "streams": 3, "status": st,
            "h2d_bytes_per_step": int(B * H * W), "d2h_bytes_per_step": int(moved["d2h"] / steps),
            "note": "copy stream: H2D of batch s+1 beside two compute streams (batches s, s-1); each batch's "
                    "compaction stores exactly the counted keypoint / descriptor / matches12 rows into host-mapped "
                    "pinned memory (orb_pack_rows_device): no D2H copy command, no host wait for counts"}


def _pcie_leg(amd, dev, m, cv, W, H, NF, B):
    """One step of B pinned host frames: H2D, extraction (+ SearchForInitialization over the B-1
    in-batch pairs when B > 1), D2H of keypoints, descriptors and matches; 10 timed steps."""
    from orb_slam2_amd import synth, _abi
    lib = _abi.lib()
    fr = np.stack([synth.frame(cv, W, H, t) for t in range(B)])
    host_in = torch.from_numpy(fr).pin_memory()
    ex = amd.ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index or 0, max_w=W, max_h=H, max_batch=B)
    cap = C.c_int()
    _abi.check("geom", lib.orb_extractor_geometry(ex._h, W, H, None, None, None, C.byref(cap)))
    cap = cap.value
    imgs = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    kps = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    m12 = torch.zeros((max(B - 1, 1), cap), dtype=torch.int32, device=dev)
    nm = torch.zeros(max(B - 1, 1), dtype=torch.int32, device=dev)
    h_kps = torch.empty(kps.shape, dtype=kps.dtype).pin_memory()
    h_desc = torch.empty(desc.shape, dtype=desc.dtype).pin_memory()
    h_m12 = torch.empty(m12.shape, dtype=m12.dtype).pin_memory()
    st = torch.cuda.current_stream(dev).cuda_stream

    def step():
        imgs.copy_(host_in, non_blocking=True)
        _abi.check("x", lib.orb_extract_batch_device(ex._h, C.c_void_p(imgs.data_ptr()), H * W, B, W, H,
                                                      C.c_void_p(kps.data_ptr()), C.c_void_p(desc.data_ptr()), cap,
                                                      C.c_void_p(cnt.data_ptr()), C.c_void_p(st)))
        if B > 1:
            _abi.check("sfi", lib.orb_search_for_initialization_batch_device(
                m._h, C.c_void_p(kps.data_ptr()), C.c_void_p(desc.data_ptr()), C.c_void_p(cnt.data_ptr()),
                C.c_void_p(kps.data_ptr() + cap * 28), C.c_void_p(desc.data_ptr() + cap * 32),
                C.c_void_p(cnt.data_ptr() + 4), B - 1, cap, W, H, 100, C.c_void_p(m12.data_ptr()),
                C.c_void_p(nm.data_ptr()), C.c_void_p(st)))
        h_kps.copy_(kps, non_blocking=True)
        h_desc.copy_(desc, non_blocking=True)
        if B > 1:
            h_m12.copy_(m12, non_blocking=True)

    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    return {"frames_per_s": round(B / dt, 1), "ms_per_step": round(dt * 1e3, 4),
            "status": batch_status(ex, m, f"PCIe-inclusive leg B={B}"),
            "h2d_bytes": int(host_in.numel()),
            "d2h_bytes": int(kps.numel() * 4 + desc.numel() + (m12.numel() * 4 if B > 1 else 0))}


class Pipe:
    """One frame sequence of the bench step: its own extractor / matcher handles, buffers and HIP
    streams, so the latency-bound stages of one sequence overlap the others on the GPU.  With
    `match_stream`, extraction and matching run on two streams of their own (a two-stage software
    pipeline over steps): SearchForInitialization of step s (match stream) overlaps the extraction
    of step s+1 (extract stream); keypoint buffers are then double-buffered by step parity, row 0
    of a buffer holding the previous step's last frame (pair t-1, t across step boundaries), copied
    on the match stream, and the extraction that next overwrites the other buffer waits for that
    copy.  tests/test_bench_pipeline.py drives this same class against the oracle."""

    def __init__(self, k, amd, dev, local, pool, W, H, NF, B, Bs, cap, match_stream=False):
        from orb_slam2_amd import _abi
        self._abi, self.lib = _abi, _abi.lib()
        self.k, self.pool, self.W, self.H, self.B, self.Bs, self.cap = k, pool, W, H, B, Bs, cap
        self.row_kp, self.row_d = cap * 28, cap * 32
        self.ts = torch.cuda.Stream(dev)
        self.tm = torch.cuda.Stream(dev) if match_stream else self.ts
        self.stream, self.mstream = self.ts.cuda_stream, self.tm.cuda_stream
        self.ex = amd.ORBextractor(NF, 1.2, 8, 20, 7, device=local, max_w=W, max_h=H, max_batch=Bs)
        self.m = amd.ORBmatcher(0.9, True, device=local)
        nb = 2 if match_stream else 1
        self.kps = [torch.zeros((Bs + 1, cap, 7), dtype=torch.int32, device=dev) for _ in range(nb)]
        self.desc = [torch.zeros((Bs + 1, cap, 32), dtype=torch.uint8, device=dev) for _ in range(nb)]
        self.counts = [torch.zeros(Bs + 1, dtype=torch.int32, device=dev) for _ in range(nb)]
        self.m12 = torch.zeros((Bs, cap), dtype=torch.int32, device=dev)
        self.nm = torch.zeros(Bs, dtype=torch.int32, device=dev)
        self.ev_ext = [torch.cuda.Event() for _ in range(2)]
        self.ev_copy = [torch.cuda.Event() for _ in range(2)]
        self.copy_pending = None
        self.last = 0

    def frame_range(self, s):
        """Pool indices of the frames step s extracts on this sequence."""
        start = (s * self.B + self.k * self.Bs) % (self.pool.shape[0] - self.Bs + 1)
        return start, start + self.Bs

    def step(self, s):
        lib, Bs, cap = self.lib, self.Bs, self.cap
        start, stop = self.frame_range(s)
        imgs = self.pool[start:stop]
        nb = len(self.kps)
        cur, prv = s % nb, (s - 1) % nb
        kps, desc, counts = self.kps[cur], self.desc[cur], self.counts[cur]
        if nb == 1:                            # one buffer: carry the last frame before overwriting
            with torch.cuda.stream(self.ts):
                kps[0].copy_(kps[Bs])
                desc[0].copy_(desc[Bs])
                counts[0:1].copy_(counts[Bs:Bs + 1])
        if self.copy_pending is not None:      # the previous step's match stream copied row Bs out
            self.ts.wait_event(self.copy_pending)
        self._abi.check("orb_extract_batch_device", lib.orb_extract_batch_device(
            self.ex._h, C.c_void_p(imgs.data_ptr()), self.H * self.W, Bs, self.W, self.H,
            C.c_void_p(kps.data_ptr() + self.row_kp), C.c_void_p(desc.data_ptr() + self.row_d), cap,
            C.c_void_p(counts.data_ptr() + 4), C.c_void_p(self.stream)))
        if nb == 2:
            self.ev_ext[s % 2].record(self.ts)
            self.tm.wait_event(self.ev_ext[s % 2])
            with torch.cuda.stream(self.tm):
                kps[0].copy_(self.kps[prv][Bs])
                desc[0].copy_(self.desc[prv][Bs])
                counts[0:1].copy_(self.counts[prv][Bs:Bs + 1])
            self.ev_copy[s % 2].record(self.tm)
            self.copy_pending = self.ev_copy[s % 2]
        self._abi.check("orb_search_for_initialization_batch_device", lib.orb_search_for_initialization_batch_device(
            self.m._h, C.c_void_p(kps.data_ptr()), C.c_void_p(desc.data_ptr()), C.c_void_p(counts.data_ptr()),
            C.c_void_p(kps.data_ptr() + self.row_kp), C.c_void_p(desc.data_ptr() + self.row_d),
            C.c_void_p(counts.data_ptr() + 4), Bs, cap, self.W, self.H, 100, C.c_void_p(self.m12.data_ptr()),
            C.c_void_p(self.nm.data_ptr()), C.c_void_p(self.mstream)))
        self.last = cur

    def status(self):
        """(extractor, matcher) overflow bits accumulated on this sequence's handles (waits for
        their streams; reading the matcher's clears it)."""
        es, ms = C.c_int32(0), C.c_int32(0)
        self.lib.orb_extractor_batch_status(self.ex._h, C.byref(es))
        self.lib.orb_matcher_batch_status(self.m._h, C.byref(ms))
        return es.value, ms.value

    def snapshot(self):
        """Host copies of the last step's outputs (call after synchronising): per extracted frame
        its keypoints / descriptors (rows 1..Bs), per pair (t-1, t) matches12 and nmatches."""
        cur = self.last
        cnt = self.counts[cur].cpu().numpy()
        kps = self.kps[cur].cpu().numpy()
        desc = self.desc[cur].cpu().numpy()
        return {"counts": cnt, "kps": kps, "desc": desc, "m12": self.m12.cpu().numpy(), "nm": self.nm.cpu().numpy()}


def bench_capacity(amd, local, W, H, NF):
    """Per-frame keypoint capacity the device batch path needs at this geometry (never truncates)."""
    from orb_slam2_amd import _abi
    ex0 = amd.ORBextractor(NF, 1.2, 8, 20, 7, device=local, max_w=W, max_h=H, max_batch=1)
    lw, lh, cells = (np.zeros(8, np.int32) for _ in range(3))
    cap = C.c_int()
    _abi.check("orb_extractor_geometry", _abi.lib().orb_extractor_geometry(
        ex0._h, W, H, _abi.ptr(lw), _abi.ptr(lh), _abi.ptr(cells), C.byref(cap)))
    return cap.value, lw, lh


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N worker processes of this script (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set) before this parent process makes any GPU
    call, forward their output and exit with the first non-zero return code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(pathlib.Path(__file__).resolve()), *sys.argv[1:]], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc != 0), 0)


def init_ranks(args):
    """Rank / device / backend of this process.  One process per GPU over RCCL ("nccl") when
    every local rank has its own device; when ranks outnumber the visible devices (a rehearsal of
    N ranks on a one-GPU lease) ranks share devices round-robin and the collectives run over gloo,
    since RCCL refuses two ranks on one device."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with torch.distributed.run "
                         f"--nproc-per-node {args.gpus}, or without a launcher (bench.py spawns the ranks)")
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("no GPU visible")
    dev_idx = local % ndev
    backend = None
    if world > 1:
        backend = "nccl" if ndev >= local_world else "gloo"
        kw = {"device_id": torch.device("cuda", dev_idx)} if backend == "nccl" else {}
        torch.distributed.init_process_group(backend, **kw)
        world = torch.distributed.get_world_size()
        rank = torch.distributed.get_rank()
    return world, rank, dev_idx, backend, min(ndev, local_world)


def main():
    args = parse()
    if os.environ.get("BENCH_STACKS_AFTER"):   # debugging aid: every thread's stack to stderr, periodically
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["BENCH_STACKS_AFTER"]), repeat=True)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world, rank, local, backend, n_devices = init_ranks(args)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # all work (torch copies, HIP kernels, collectives) on one explicit non-default stream
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    amd = pkgload.load()
    from orb_slam2_amd import _abi, synth

    W, H, B, NF = args.width, args.height, args.batch, args.nfeatures
    # ---- synthetic stream resident in HBM (seed per rank: shards are independent streams)
    cv = synth.canvas(0x5EED0002 + 1000 * rank, W, H)
    pool_np = np.stack([synth.frame(cv, W, H, t) for t in range(max(args.pool, B))])
    pool = torch.from_numpy(pool_np).to(dev)
    S = max(1, min(args.streams, B))
    assert B % S == 0, "--batch must be a multiple of --streams"
    Bs = B // S

    cap, lw, lh = bench_capacity(amd, local, W, H, NF)
    lib = _abi.lib()
    torch.cuda.synchronize(dev)
    pipes = [Pipe(k, amd, dev, local, pool, W, H, NF, B, Bs, cap, args.match_stream) for k in range(S)]
    ex = pipes[0].ex

    def step(s):
        for p in pipes:
            p.step(s)

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(args.warmup + s)
    t_enq = time.perf_counter() - t0   # host time to enqueue the K steps (the GPU runs behind it)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    # overflow bits of every sequence's extractor and matcher over warm-up + timed steps: a set bit
    # means some frame's keypoints or some pair's candidate list were truncated (not the reference)
    ext_status = mat_status = 0
    for p in pipes:
        e, m = p.status()
        ext_status |= e
        mat_status |= m
    if ext_status or mat_status:
        raise SystemExit(f"bench: overflow status extractor={ext_status} matcher={mat_status}")
    # per-kernel launch spans under the streams' sharing: a few more steps after the timed region
    # with HIP events at every stream's four extraction kernels' boundaries (k_pyramid, k_fast_cell,
    # k_octree, k_orient_desc: five events per call, mode 3) on its launch stream — kept out of the
    # timed region, whose steps carry no instrumentation
    n_shared = 4
    if not args.no_profile:
        for p in pipes:
            lib.orb_extractor_profile(p.ex._h, 3)
        for s in range(n_shared):
            step(args.warmup + args.steps + s)
        torch.cuda.synchronize(dev)

    def stage_times():
        tot, calls = np.zeros(6), 0
        for p in pipes:
            sm, nc = np.zeros(6), C.c_int(0)
            lib.orb_extractor_stage_times(p.ex._h, _abi.ptr(sm), 6, C.byref(nc))
            lib.orb_extractor_profile(p.ex._h, 0)
            tot += sm
            calls += nc.value
        return tot, calls
    stage_ms, nstage = stage_times() if not args.no_profile else (np.zeros(6), 0)
    iso_ms = None
    if not args.no_profile:
        # the isolated pass: sequence 0's step (one 128-frame extraction launch + its matching) alone
        # on its stream, kernels serialised, HIP events at the extraction kernels' boundaries — the
        # live counterpart of the committed rocprofv3 summary ISOLATED_STATS
        p0, n_iso = pipes[0], 10
        lib.orb_extractor_profile(p0.ex._h, 3)
        torch.cuda.synchronize(dev)
        for s in range(n_iso):
            p0.step(args.warmup + args.steps + n_shared + s)
        torch.cuda.synchronize(dev)
        sm, nc = np.zeros(6), C.c_int(0)
        lib.orb_extractor_stage_times(p0.ex._h, _abi.ptr(sm), 6, C.byref(nc))
        lib.orb_extractor_profile(p0.ex._h, 0)
        iso_ms = sm / max(nc.value, 1)
    frames_total = B * args.steps * world
    value = frames_total / dt
    cnt = torch.cat([p.counts[p.last][1:] for p in pipes]).cpu().numpy()
    nmatch = torch.cat([p.nm for p in pipes]).cpu().numpy()

    result = {
        "metric": "frames/sec ORB extract+match @640x480; local-BA ms/iter",
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "world_size": world,
        "collective_backend": backend,
        "distinct_devices": n_devices if world > 1 else 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * dt / args.steps, 4),
        "host_enqueue_ms_per_step": round(1000 * t_enq / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"synthetic {W}x{H} grayscale stream, {NF} feat/frame, 8 levels, scale 1.2, "
                               f"FAST 20/7; extract + SearchForInitialization(t-1,t; window 100, nnratio 0.9, "
                               f"checkOri) per frame; {B} frames per step per GPU as {S} independent "
                               f"sequences, each on its own HIP stream"
                               f"{' plus a matching stream (matching of step s overlaps extraction of step s+1)' if args.match_stream else ' (extraction then matching)'}"
                               f", HBM-resident",
                   "batch_per_gpu": B, "streams_per_gpu": S, "width": W, "height": H, "nfeatures": NF,
                   "parallelism": f"frame-sharded x{world}"},
        "status": {"extractor": ext_status, "matcher": mat_status},
        "keypoints_per_frame": float(np.mean(cnt)),
        "matches_per_pair": float(np.mean(nmatch)),
    }
    progress(rank, f"extraction + matching timed: {value:.0f} frames/s")
    pre = np.zeros(8, np.int32)
    lib.orb_extractor_last_counts(ex._h, 0, _abi.ptr(pre), None)
    n_pre_frame = float(pre.sum())   # corners k_fast_cell emitted for frame 0 of the last batch
    copy_peak = measure_copy_peak(dev)
    if nstage > 0:
        result["roofline"] = extraction_roofline(stage_ms, nstage, lw, lh, n_pre_frame, float(np.mean(cnt)), W, H, NF,
                                                 Bs, iso_ms=iso_ms, launches_per_step=S,
                                                 ms_per_step=result["ms_per_step"])
        if result["roofline"]:
            result["roofline"]["hbm"]["measured_copy_peak_gbs"] = copy_peak
            result["roofline"]["hbm"]["frac_of_measured_copy_peak"] = round(
                result["roofline"]["hbm"]["achieved"] / copy_peak, 5)
    if nstage > 0:
        result["stage_ms_per_batch"] = {k: round(float(v) / nstage, 4) for k, v in zip(STAGES, stage_ms)
                                        if not k.startswith("reserved")}
        result["stage_ms_source"] = (f"{n_shared} steps after the timed region, the same {S} streams: HIP events at the "
                                     "kernel boundaries on each stream, average launch span while the other streams' "
                                     "kernels share the chip (not a kernel's own duration; the isolated durations are "
                                     "roofline.kernels[*].isolated_launch_ms)")
    if iso_ms is not None:
        result["stage_ms_isolated_live"] = {k: round(float(v), 4) for k, v in zip(STAGES, iso_ms)
                                            if not k.startswith("reserved")}
    # whole-pipeline roofline of SURVEY §8d: B_ext = P0 + 2 sum_{l>=1} P_l + N_kp (28 + 32) per frame
    P = (lw.astype(np.int64) * lh)
    b_ext = float(P[0] + 2 * P[1:].sum()) + float(np.mean(cnt)) * 60.0
    result["pipeline_roofline"] = {"bytes_per_frame": b_ext, "achieved_gbs": round(b_ext * value / 1e9, 2),
                                   "peak_gbs": HBM_PEAK_GBS, "frac": round(b_ext * value / 1e9 / HBM_PEAK_GBS, 5),
                                   "measured_copy_peak_gbs": copy_peak,
                                   "frac_of_measured_copy_peak": round(b_ext * value / 1e9 / copy_peak, 5),
                                   "copy_peak_source": "1 GiB device-to-device torch copy x8 in this run (read + write bytes)",
                                   "pmc_capture_matches_tree": pmc_capture_current()}
    # the whole step against the VALU bound: every extraction + matching kernel's lane-ops per
    # frame (committed PMC pass of this configuration) x frames/s
    kern = ("k_pyramid", "k_fast_cell", "k_octree", "k_orient_desc", "k_grid_sfi", "k_cand_sfi", "k_resolve_sfi")
    ops = [pmc_valu_ops(k, W, H, NF, Bs) for k in kern]
    if all(o is not None for o in ops):
        per_frame = sum(ops) / Bs
        ach = per_frame * value / 1e12
        alg_frame = sum(algorithmic_ops(st, lw, lh, float(n_pre_frame), float(np.mean(cnt)))
                        for st in ("resize", "fast_detect", "octree", "orient_blur_desc"))
        result["pipeline_algorithmic"] = {"ops_per_frame": int(alg_frame), "achieved": round(alg_frame * value / 1e12, 3),
                                          "unit": "TOP/s", "peak": VALU_PEAK_TOPS,
                                          "frac": round(alg_frame * value / 1e12 / VALU_PEAK_TOPS, 4),
                                          "issued_lane_ops_per_algorithmic_op": round(per_frame / max(alg_frame, 1), 2),
                                          "model": "ALG_OPS in bench.py (extraction stages; the matcher not counted)"}
        result["pipeline_valu"] = {"lane_ops_per_frame": round(per_frame), "kernels": list(kern),
                                   "achieved": round(ach, 3), "unit": "TOP/s", "peak": VALU_PEAK_TOPS,
                                   "frac": round(ach / VALU_PEAK_TOPS, 4), "measured_issue_peak": VALU_MEASURED_TOPS,
                                   "frac_of_measured_issue_peak": round(ach / VALU_MEASURED_TOPS, 4),
                                   "frac_of_measured_f32_issue_peak": round(ach / VALU_MEASURED_F32_TOPS, 4),
                                   "ops_source": PMC_VALU.name}
    if not args.no_lba:
        progress(rank, "local BA (config 4)")
        result["lba"] = bench_lba(args, amd, dev, local, rank, world)
        if not args.no_lba_scaled:
            progress(rank, "local BA, scaled windows")
            result["lba_scaled"] = bench_lba_scaled(args, amd, dev, rank, world)
    if not args.no_stereo:
        progress(rank, "config 5 (stereo)")
        result["config5_stereo_sharded"] = bench_config5(args, amd, dev, rank, world)
    if world == 1 and not args.no_extras:
        progress(rank, "extras")
        result["extras"] = bench_extras(args, amd, dev)
    if world == 1 and not args.no_cpu:   # rank 0 at N=1 only
        progress(rank, "CPU baseline (extraction + matching)")
        result["cpu_baseline"] = cpu_baseline(pool_np[: min(len(pool_np), 512)], NF, args.cpu_seconds)
        result["speedup_vs_cpu_baseline"] = round(value / result["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
