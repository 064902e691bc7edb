#!/usr/bin/env python3
"""Benchmark: Msamples/s + achieved bytes/s of the render kernel on the RTOW final scene.

One step = one whole frame of BASELINE config 2 (rtweekend_final_image scene at set_seed(42),
1200x800, 500 spp, max_depth 50) rendered by the gfx950 kernel from a scene already resident in
HBM. With N ranks (torchrun, one process per GPU) the frame's rows are dealt to ranks in 4-row
blocks, each rank renders its blocks, and the tiles are all-gathered over RCCL (xGMI) into a full
frame on every rank: the total work is fixed, so scaling is "strong". The gather of frame i runs
on a side stream while frame i + 1 renders (double-buffered frames).

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N ranks
itself (torch.distributed.run, 127.0.0.1) before anything touches a GPU, and fails when fewer than
N GPUs are visible; under a launcher (WORLD_SIZE set) it is one rank.

Prints ONE JSON line on rank 0 (see the repo contract), with
  roofline:     the resource that binds the render kernel. The scene is LDS/L2-resident and the
                kernel moves ~7 GB per launch to/from HBM (~1% of peak), so the bound is VALU
                issue: bound "valu", frac = the share of SIMD cycles the VALU issue port is busy
                in the timed kernel, from the rocprofv3 PMC passes of this exact build
                (profiles/pmc_latest.json: 4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) /
                SIMD cycles, i.e. VALU issue quad-cycles net of gfx950 dual issue; the older
                instruction-class model is kept beside it), lane_util = active lanes per VALU
                instruction. The HBM figures are reported beside it, labelled: `hbm.algorithmic`
                = SURVEY 8d bytes (56 B per BVH node visited, 36 B per sphere test, 124 B per
                parallelogram test, 24 B per pixel written; visit counts from an untimed
                instrumented pass) / kernel time — bytes the path touches, almost all served by
                LDS and L1/L2, so its "fraction" may exceed 1 — and `hbm.measured` = PMC HBM bytes
                (FETCH_SIZE x2 + WRITE_SIZE) / kernel time against the 8 TB/s peak.
  cpu_baseline: the reference's own Camera::render (oracle/_ref, built from the reference
                sources) on the host, as BASELINE.md §3 specifies: the same frame (config 2
                whole, 500 spp; configs 3-5 at a reduced --cpu-spp, extrapolated linearly in
                samples and labelled so), threads = the CPUs this process is granted (usable CPUs
                capped at the cgroup CPU quota: 16 on the GPU box), median of 3 runs; CPU model,
                host CPU count and quota reported, and an oversubscribed one-run figure (every
                affinity CPU a thread) beside it, labelled secondary.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X spec (vector FP64)
NODE_B, SPHERE_B, QUAD_B, PIXEL_B = 56, 36, 124, 24
SCENE_DATA = {
    "rtow_final": "synthetic: rtweekend_final_image scene built by the reference's RNG at set_seed(42)",
    "cornell": "synthetic: cornell_box_test(false) scene of the reference's src/main.cpp (no randomness)",
    "millions": "synthetic: millions_of_spheres scene built by the reference's RNG at set_seed(42)",
}


def build_stamp() -> dict:
    """The loaded library's build stamp (crt_build_info: its compile-time switches, the sha256 of
    its sources as compiled and their git commit, '+dirty' when they were not committed)."""
    import cpp_raytracer_amd as crt
    info = crt.lib().crt_build_info().decode()
    kv = dict(x.split("=", 1) for x in info.split() if "=" in x)
    git = kv.get("git", "none")
    return {"build_info": info, "source_sha": kv.get("src", "unknown"), "git_commit": git.split("+")[0],
            "git_dirty": git.endswith("+dirty") or git == "none"}


def kernel_source_sha() -> str:
    """Hash of the loaded library's build info without its git field (its switches and the sha of
    the sources it was compiled from, baked in by the Makefile): a PMC summary
    (profiles/pmc_latest.json) is used only when it was collected on a build of these exact
    sources; the commit is recorded beside it (and must be clean), but later commits that do not
    touch the library's sources leave the match intact."""
    import hashlib
    info = " ".join(x for x in build_stamp()["build_info"].split() if not x.startswith("git="))
    return hashlib.sha256(info.encode()).hexdigest()[:16]


def pmc_summary_usable(pj: dict, workload: str) -> bool:
    """A PMC summary describes this run's kernel only when it was collected on this exact build of
    a committed tree (tools/gpu_pmc.sh refuses dirty builds and records the commit) for this
    workload; a hand-edited one (sha_note) never is."""
    return (pj.get("workload") == workload and pj.get("kernel_source_sha") == kernel_source_sha()
            and "sha_note" not in pj and pj.get("git_dirty") is False and bool(pj.get("git_commit")))


def cgroup_cpu_quota() -> float | None:
    """CPUs' worth of time the cgroup grants this process (cpu.max quota / period), or None."""
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = Path(p).read_text().split()[:2]
            if q != "max":
                return round(int(q) / int(per), 2)
        except (OSError, ValueError):
            pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        return round(q / per, 2) if q > 0 else None
    except (OSError, ValueError):
        return None


def cpu_info() -> tuple[str, int, int]:
    """(CPU model, host CPUs, CPUs this process may use)."""
    model = "unknown"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return model, os.cpu_count() or 1, usable


def self_launch(args) -> int:
    """Run this script as N ranks (one per GPU) under torch.distributed.run and return its exit
    code. Called before any GPU initialisation (torch.cuda.device_count() does not initialise
    HIP on this image)."""
    import socket
    import torch
    if not args.launch_check:
        visible = torch.cuda.device_count()
        if visible < args.gpus:
            print(f"[bench] --gpus {args.gpus} but only {visible} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *sys.argv[1:]]
    return subprocess.run(cmd).returncode


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="rtow_final")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--base-seed", type=int, default=2024)
    ap.add_argument("--cpu-spp", type=int, default=0,
                    help="spp of the CPU-baseline frame (0 = the benchmarked spp: BASELINE.md §3 runs config 2 "
                         "whole; configs 3-5 run reduced spp, extrapolated linearly in samples)")
    ap.add_argument("--cpu-runs", type=int, default=3, help="CPU-baseline runs (the median is reported)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the CPUs this process is granted: usable CPUs capped at the cgroup quota")
    ap.add_argument("--cpu-share-spp", type=int, default=100,
                    help="spp of the secondary, oversubscribed one-run figure (every affinity CPU a thread); 0 = skip")
    ap.add_argument("--launch-check", action="store_true",
                    help="ranks only join the process group and report (tests the N-rank launch on CPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dump-frame", default="", help="save every rank's last assembled frame to PATH.rank<r>.npy")
    ap.add_argument("--pmc-json", default=str(ROOT / "profiles" / "pmc_latest.json"))
    return ap.parse_args()


def baseline_threads(args) -> tuple[int, str]:
    """Threads of the CPU baseline: --cpu-threads, else the CPUs this process is granted: the
    usable (affinity) CPUs, capped at the cgroup's CPU quota when there is one (on the GPU box the
    affinity mask lists 256 CPUs but the cgroup grants 16 CPUs' worth of time: 256 threads would
    only oversubscribe those 16)."""
    _, _, usable = cpu_info()
    if args.cpu_threads:
        return args.cpu_threads, "--cpu-threads"
    quota = cgroup_cpu_quota()
    if quota is not None and int(quota) < usable:
        return max(1, int(quota)), f"cgroup CPU quota {quota} (affinity lists {usable} CPUs)"
    return usable, "usable (affinity) CPUs"


def cpu_baseline(args, scene_data, log) -> dict | None:
    """The reference's own Camera::render on the host (oracle/_ref, built from the reference
    sources; camera.h:301-303 = render<BVH>(BVH(world)), OpenMP rows, its own per-thread RNG), as
    BASELINE.md §3 specifies: the same scene and image, threads = the CPUs this process is granted
    (baseline_threads), median of --cpu-runs runs. With --cpu-spp below the benchmarked spp (the
    frames of configs 3-5, BASELINE.md §3 "Coverage") the render loop's rate is measured on that
    reduced-spp frame and extrapolated linearly in samples; the BVH build is timed apart and
    counted once per frame. A secondary one-run figure with every affinity CPU as a thread is kept,
    labelled, when that differs (oversubscribed)."""
    import statistics
    import cpp_raytracer_amd as crt
    from cpp_raytracer_amd import camera_with
    model, host_cpus, usable = cpu_info()
    threads, basis = baseline_threads(args)
    ref = ROOT / "oracle" / "_ref" / "ref_driver"
    runs = max(1, args.cpu_runs)
    spp = min(args.cpu_spp or args.spp, args.spp)
    full_samples = args.width * args.height * args.spp
    extrapolated = spp < args.spp
    host = {"cpu_model": model, "host_cpus": host_cpus, "usable_cpus": usable, "cgroup_cpu_quota": cgroup_cpu_quota(),
            "threads_basis": basis}

    def frame(n_spp):
        return crt.SceneData(scene_data.materials, scene_data.objects,
                             camera_with(scene_data.camera, image_w=args.width, image_h=args.height,
                                         samples_per_pixel=n_spp, max_depth=args.depth))

    def desc(n_spp, n_runs):
        return (f"{args.scene} seed {args.seed}, {args.width}x{args.height}, {n_spp} spp, depth {args.depth}"
                + (f"; median of {n_runs} runs" if n_runs > 1 else "; one run"))

    def summary(rates, builds, kind, sample):
        rate = statistics.median(rates)
        build = statistics.median(builds) if builds else 0.0
        out = {"value": round(rate, 4), "unit": "Msamples/s", "cores": threads, "kind": kind,
               "runs": [round(x, 4) for x in rates], **host, "sample": sample,
               "extrapolated": extrapolated}
        if builds:
            out["bvh_build_seconds"] = round(build, 4)
        if extrapolated:
            out["extrapolation"] = (f"render-loop rate of the {spp}-spp frame, linear in samples to the "
                                    f"benchmarked {args.spp} spp (BASELINE.md §3 Coverage)")
        out["frame_seconds"] = round(full_samples / (rate * 1e6) + build, 3)
        return out

    with tempfile.TemporaryDirectory() as td:
        def ref_runs(n_spp, n_threads, n_runs):
            p = Path(td) / f"scene_{n_spp}.crts"
            if not p.exists():
                frame(n_spp).save(p)
            rates, builds = [], []
            for _ in range(n_runs):
                r = subprocess.run([str(ref), "time", str(p), str(n_threads)], capture_output=True, text=True,
                                   timeout=900, check=True)
                j = json.loads(r.stdout.strip().splitlines()[-1])
                rates.append(j["samples"] / j["seconds"] / 1e6)
                builds.append(j.get("build_seconds", 0.0))
            return rates, builds

        if ref.exists():
            try:
                rates, builds = ref_runs(spp, threads, runs)
                out = summary(rates, builds, "reference",
                              desc(spp, runs) + " (reference render<BVH>(BVH(world)), OpenMP, own per-thread RNG)")
                if usable > threads and args.cpu_share_spp:
                    r2, _ = ref_runs(min(args.cpu_share_spp, spp), usable, 1)
                    out["oversubscribed"] = {
                        "value": round(r2[0], 4), "unit": "Msamples/s", "cores": usable,
                        "sample": desc(min(args.cpu_share_spp, spp), 1) + f" with {usable} threads (every "
                        "affinity CPU); secondary, not the baseline: the cgroup grants fewer CPUs' time"}
                return out
            except Exception as e:  # pragma: no cover - reported, not fatal
                log(f"reference CPU baseline failed: {e}")
        try:
            sys.path.insert(0, str(ROOT / "oracle"))
            import crt_oracle_py as orc
            d = frame(spp)
            rates = []
            for _ in range(runs):
                secs, n = orc.time_render(d, threads, args.base_seed)
                rates.append(n / secs / 1e6)
            return summary(rates, [], "port", desc(spp, runs) + " (oracle C restatement, OpenMP)")
        except Exception as e:  # pragma: no cover
            log(f"port CPU baseline failed: {e}")
    return None


DIGESTS = ROOT / "tests" / "golden" / "frame_digests.json"


def frame_check(workload: str, base_seed: int, digest: str, agree: bool, rank_digests: list, world: int) -> dict:
    """The bench line's frame self-check: rank 0's frame digest, whether every rank assembled the
    same frame, and whether it equals the N=1 digest recorded for this workload and base seed
    (tests/golden/frame_digests.json, from a one-GPU run; null when none is recorded)."""
    key = f"{workload}; base_seed {base_seed}"
    try:
        recorded = json.loads(DIGESTS.read_text()).get(key)
    except (OSError, ValueError):
        recorded = None
    return {"frame_digest": digest, "ranks_agree": agree, "rank_digests": rank_digests if world > 1 else None,
            "recorded_n1_digest": recorded, "matches_n1": (digest == recorded) if recorded else None,
            "basis": "sha256 of the assembled float64 frame (first 15 hex digits), every rank; frames are "
                     "bit-identical for any rank count"}


def launch_check(args) -> int:
    """One rank of `--launch-check`: join the process group (gloo, CPU), agree on the world size
    with an all-reduce, rank 0 prints it."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.ones(1)
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"launch_check": True, "world_size": dist.get_world_size(), "all_reduce": float(t[0]),
                          "requested": args.gpus}), flush=True)
    dist.destroy_process_group()
    return 0


def main() -> int:
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return self_launch(args)
    if args.launch_check:
        return launch_check(args)
    import torch
    import torch.distributed as dist
    import cpp_raytracer_amd as crt
    from cpp_raytracer_amd import Tiling, camera_with
    from cpp_raytracer_amd.tiles import TileGather, digests_agree, frame_digest, owned_rows

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: reporting the {world} ranks that run",
              file=sys.stderr, flush=True)
    distributed = world > 1
    # one GPU per rank; CRT_BENCH_BACKEND=gloo + ranks sharing a device rehearses the N>1 path
    # on a one-GPU box (RCCL refuses two ranks on one device)
    backend = os.environ.get("CRT_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if distributed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    t0 = time.time()
    data = crt.SceneData.named(args.scene, args.seed)
    data.camera = camera_with(data.camera, image_w=args.width, image_h=args.height,
                              samples_per_pixel=args.spp, max_depth=args.depth)
    ts = time.perf_counter()
    scene = crt.GpuScene(data, build_device=local if len(data.objects) > 100000 else None)
    info = scene.info()
    scene.upload(local)
    setup_ms = (time.perf_counter() - ts) * 1e3  # flattening, BVH build, staging, upload (untimed)
    cam = crt.resolve_camera(data.camera, args.base_seed)
    h, w = args.height, args.width
    rb = 4  # 4-row blocks: 800 rows deal exactly over 1, 2, 4, 8 ranks (16 left 7 vs 6 at N=8)
    tiling = Tiling(rb, world, rank, 0)
    owned = owned_rows(h, rb, world, rank)
    log(f"scene {args.scene}: {info.num_primitives} prims, {info.num_nodes} nodes, depth {info.depth}, "
        f"BVH build {info.build_ms:.1f} ms, setup {time.time() - t0:.1f} s")

    gather = TileGather(h, w, world, rank, "cuda", row_block=rb)
    # N > 1: each rank renders its rows only, packed in order into a tile of its share
    # (CRT_TILING_PACKED), which is also the all-gather's input: no full-frame buffer per rank
    if distributed:
        tiling = Tiling(rb, world, rank, 1)
        frames = [gather.new_tile() for _ in range(2)]
    else:
        frames = [torch.zeros(h, w, 3, dtype=torch.float64, device="cuda")]
    stream = torch.cuda.current_stream()
    side = torch.cuda.Stream() if distributed else None
    gathered = [None] * len(frames)  # per frame buffer: event after its last gather
    assembled = [None]  # the last assembled frame (--dump-frame)

    def step(i, ev=None):
        # N > 1: frame i's tiles are all-gathered (RCCL over xGMI) on a side stream while frame
        # i + 1 renders into the other buffer; a buffer is rendered into again only after its
        # previous gather is done. Every frame is rendered AND assembled inside the timed region.
        k = i % len(frames)
        buf = frames[k]
        if gathered[k] is not None:
            stream.wait_event(gathered[k])
        if ev is not None:
            ev[0].record(stream)
        scene.render_async(local, cam, buf.data_ptr(), stream.cuda_stream, tiling)
        if ev is not None:
            ev[1].record(stream)
        if distributed:
            rendered = torch.cuda.Event()
            rendered.record(stream)
            with torch.cuda.stream(side):
                side.wait_event(rendered)
                assembled[0] = gather.gather_packed(buf)
                done = torch.cuda.Event()
                done.record(side)
            gathered[k] = done
        else:
            assembled[0] = buf

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, evs[i])
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / max(1, args.steps)
    if args.dump_frame:  # every rank's last assembled frame (tests: equal to the 1-rank frame)
        import numpy as np
        np.save(f"{args.dump_frame}.rank{rank}.npy", assembled[0].cpu().numpy())
    # self-check of the assembled frame (untimed): every rank hashes the frame it holds, the digests
    # are all-gathered, and rank 0 compares them with each other and with the recorded N=1 digest
    # of this workload (frames are bit-identical for any rank count). CRT_BENCH_CORRUPT_RANK=k
    # (tests only) flips one value of rank k's frame first, which must flip ranks_agree.
    final = assembled[0]
    if os.environ.get("CRT_BENCH_CORRUPT_RANK", "") == str(rank):
        final = final.clone()
        final.view(-1)[final.numel() // 2] += 1.0
    digest = frame_digest(final)
    if distributed:
        agree, rank_digests = digests_agree(digest, "cuda" if dist.get_backend() == "nccl" else "cpu")
    else:
        agree, rank_digests = True, [digest]
    if distributed:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])
    samples_total = h * w * args.spp * args.steps
    ms_per_step = elapsed * 1e3 / max(1, args.steps)

    # algorithmic bytes of one launch (this rank's tile), from the instrumented pass (untimed),
    # which walks like the reference (its node counts are the byte basis); a second instrumented
    # pass walks speculatively like the timed kernel (CRT_COUNT_SPEC=1, read at the call) for the
    # timed kernel's phase shares and lane utilization
    cnt = scene.render_count(local, cam, tiling)
    os.environ["CRT_COUNT_SPEC"] = "1"
    try:
        cnt_spec = scene.render_count(local, cam, tiling)
    finally:
        del os.environ["CRT_COUNT_SPEC"]
    alg_bytes = (cnt.nodes_visited * NODE_B + cnt.sphere_tests * SPHERE_B + cnt.parallelogram_tests * QUAD_B
                 + len(owned) * w * PIXEL_B)
    rays_per_sample = cnt.rays / max(1, cnt.samples)
    flops = cnt.nodes_visited * 12 + cnt.sphere_tests * 23 + cnt.parallelogram_tests * 40 + cnt.rays * 50
    achieved_gbs = alg_bytes / (kernel_ms * 1e-3) / 1e9
    workload = f"{args.scene} seed {args.seed}, {w}x{h}, {args.spp} spp, max_depth {args.depth}"
    if (args.scene, w, h, args.spp, args.depth) == ("rtow_final", 1200, 800, 500, 50):
        workload += " (BASELINE config 2)"
    # counters of the timed kernel from the rocprofv3 PMC passes (tools/gpu_pmc.sh +
    # tools/pmc_summary.py) of this workload on this exact build
    pmc_data, pmc_src = None, None
    # --pmc-json first, then the per-config summaries beside it (profiles/pmc_c<k>.json)
    pmc_paths = [Path(args.pmc_json)] + sorted(Path(args.pmc_json).parent.glob("pmc_c*.json"))
    for pmc in pmc_paths if world == 1 else []:
        try:
            pj = json.loads(pmc.read_text())
        except Exception:
            continue
        if pmc_summary_usable(pj, workload):
            pmc_data = pj
            pmc_src = str(pmc.relative_to(ROOT)) if pmc.is_relative_to(ROOT) else str(pmc)
            break
    traffic = pmc_data.get("hbm_bytes_per_launch") if pmc_data else None
    measured_gbs = traffic / (kernel_ms * 1e-3) / 1e9 if traffic else None
    issue = pmc_data.get("valu_issue_frac") if pmc_data else None
    roofline = {
        "bound": "valu",
        "achieved": round(issue, 4) if issue is not None else None,
        "peak": 1.0,
        "unit": "VALU issue-busy cycles per SIMD cycle",
        "frac": round(issue, 4) if issue is not None else None,
        "traffic": traffic,
        "lane_util": round(pmc_data["valu_lane_utilization"], 4) if pmc_data and "valu_lane_utilization" in pmc_data else None,
        "valu_basis": (pmc_data.get("valu_issue_basis") if pmc_data else None),
        "valu_frac_simple_model": (round(pmc_data["valu_issue_frac_model"], 4)
                                   if pmc_data and "valu_issue_frac_model" in pmc_data else None),
        "valu_frac_class_model": (round(pmc_data["valu_issue_frac_class_model"], 4)
                                  if pmc_data and "valu_issue_frac_class_model" in pmc_data else None),
        "valu_dual_issue_share": (round(pmc_data["valu_dual_issue_share"], 4)
                                  if pmc_data and "valu_dual_issue_share" in pmc_data else None),
        "waves_per_simd": (round(pmc_data["avg_waves_per_simd"], 2)
                           if pmc_data and "avg_waves_per_simd" in pmc_data else None),
        "valu_costs": "SIMD cycles = 32 x SQ_BUSY_CYCLES (1024 SIMDs), cross-checked against GRBM_GUI_ACTIVE; "
                      "class model: per-instruction costs measured by tools/valu_rate.hip",
        "pmc_source": pmc_src,
        "kernel_ms": round(kernel_ms, 3),
        "hbm": {
            "peak_GBps": HBM_PEAK_GBS,
            "algorithmic": {"GBps": round(achieved_gbs, 1), "frac_of_peak": round(achieved_gbs / HBM_PEAK_GBS, 4),
                            "bytes_per_launch": int(alg_bytes),
                            "basis": "SURVEY 8d bytes the path touches (56 B/node, 36 B/sphere test, 124 B/quad "
                                     "test, 24 B/pixel); served almost entirely by LDS and L1/L2, not HBM"},
            "measured": {"GBps": round(measured_gbs, 1) if measured_gbs else None,
                         "frac_of_peak": round(measured_gbs / HBM_PEAK_GBS, 4) if measured_gbs else None,
                         "bytes_per_launch": traffic,
                         "basis": "rocprofv3 PMC: 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section)"},
        },
    }
    # the honest pair beside the issue-port figure: useful f64 work against the vector f64 peak,
    # and issue-busy weighted by the share of lanes active per instruction
    fp64_tflops = flops / (kernel_ms * 1e-3) / 1e12
    roofline["useful_frac"] = round(fp64_tflops / FP64_VECTOR_PEAK_TFLOPS, 4)
    roofline["useful_basis"] = ("algorithmic f64 flops (12 per node test, 23 per sphere test, 40 per "
                                "parallelogram test, 50 per ray) / kernel time / 78.6 TF vector f64 peak")
    roofline["lane_weighted_issue"] = (round(issue * pmc_data["valu_lane_utilization"], 4)
                                       if issue is not None and "valu_lane_utilization" in pmc_data else None)
    if pmc_data is None:
        roofline["note"] = ("no PMC summary of this workload on this exact committed build (tools/gpu_pmc.sh): "
                            "issue fraction and traffic unmeasured")

    # Dielectric reflect-or-refract draws of every rendered frame (warm-up, timed, instrumented)
    # that a one-ulp different pow() could have flipped (crt_schlick.h): 0 = every branch is the
    # reference's whatever libm the reference is built against
    guard = scene.guard(local)
    if distributed:
        t = torch.tensor([alg_bytes, cnt.rays, cnt.samples, cnt.nodes_visited, guard], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)  # totals for the record
        guard = int(t[4])
    if rank == 0:
        cpu = None if args.no_cpu_baseline else cpu_baseline(args, data, log)
        out = {
            "metric": "Msamples/sec + achieved HBM GB/s, RTOW final scene at 1/2/4/8 MI355X",
            "value": round(samples_total / elapsed / 1e6, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": SCENE_DATA.get(args.scene, f"synthetic: {args.scene} scene of the reference's src/main.cpp"),
            "config": {"workload": workload,
                       "samples_per_step": h * w * args.spp, "primitives": int(info.num_primitives),
                       "bvh_nodes": int(info.num_nodes), "scene_setup_ms": round(setup_ms, 1), "partition": f"{rb}-row blocks over {world} ranks, "
                       "RCCL all-gather of tiles overlapped with the next frame" if distributed else "whole frame on one GPU",
                       "process_group": {"backend": dist.get_backend() if distributed else None,
                                         "world_size": dist.get_world_size() if distributed else 1,
                                         "visible_gpus": torch.cuda.device_count()}},
            "roofline": roofline,
            "fp64": {"achieved_tflops": round(flops / (kernel_ms * 1e-3) / 1e12, 3),
                     "peak_tflops": FP64_VECTOR_PEAK_TFLOPS, "rays_per_sample": round(rays_per_sample, 4),
                     "nodes_per_ray": round(cnt.nodes_visited / max(1, cnt.rays), 3),
                     "prim_tests_per_ray": round((cnt.sphere_tests + cnt.parallelogram_tests) / max(1, cnt.rays), 3)},
            # per-phase shares and lane utilization of the two instrumented passes: the timed
            # kernel's (speculative walk) and the reference-like one (plain walk, whose node
            # counts are the byte basis)
            "instrumented_pass": {"timed_walk": "speculative walk, as the timed kernel (CRT_COUNT_SPEC=1)",
                                  "plain_walk": "reference node-test sequence (algorithmic-byte basis)"},
            "wave_time_share": {k: round(getattr(cnt_spec, "ticks_" + k) / max(1, cnt_spec.ticks_total), 4)
                                for k in ("walk", "leaf", "shade", "tail")},
            "lane_utilization": {
                "walk": round(cnt_spec.nodes_visited / max(1, 64 * cnt_spec.wave_iters_walk), 4),
                "leaf": round((cnt_spec.sphere_tests + cnt_spec.parallelogram_tests) / max(1, 64 * cnt_spec.wave_iters_leaf), 4),
                "shade": round(cnt_spec.rays / max(1, 64 * cnt_spec.wave_iters_shade), 4)},
            "lane_utilization_plain_walk": {
                "walk": round(cnt.nodes_visited / max(1, 64 * cnt.wave_iters_walk), 4),
                "leaf": round((cnt.sphere_tests + cnt.parallelogram_tests) / max(1, 64 * cnt.wave_iters_leaf), 4),
                "shade": round(cnt.rays / max(1, 64 * cnt.wave_iters_shade), 4)},
            "two_pass_leaves": {"candidates_per_ray": round(cnt.candidate_tests / max(1, cnt.rays), 4),
                                "candidate_lane_utilization": round(cnt.candidate_tests / max(1, 64 * cnt.wave_iters_candidates), 4),
                                "candidate_wave_iters_per_filter_wave_iter": round(cnt.wave_iters_candidates / max(1, cnt.wave_iters_leaf), 4)},
            "f32_walk": {"f64_decided_node_tests": round(cnt.slow_node_tests / max(1, cnt.nodes_visited), 6),
                         "walk_iters_with_f64": round(cnt.wave_iters_slow / max(1, cnt.wave_iters_walk), 6)},
            # raw counts of both instrumented passes (wave iterations per phase, lanes' tests):
            # the basis of DESIGN §5's per-phase VALU attribution (tools/valu_attribution.py)
            "instrumented_counts": {name: {f: int(getattr(c, f)) for f, _ in c._fields_ if f != "kernel_ms"}
                                    for name, c in (("timed_walk", cnt_spec), ("plain_walk", cnt))},
            "schlick_guard": {"undecided_draws": guard, "frames": args.warmup + args.steps + 2,
                              "basis": "Dielectric draws a one-ulp different pow() could flip, counted by the "
                                       "kernel (crt_render_guard); 0 = frames bit-for-bit the reference's branches"},
            "cpu_baseline": cpu,
            "frame_check": frame_check(workload, args.base_seed, digest, agree, rank_digests, world),
        }
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
