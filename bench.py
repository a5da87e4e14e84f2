#!/usr/bin/env python3
"""Benchmark: Msamples/s (paths/s) on CornellBox 1024^2, depth 8 (BASELINE.json configs[1]).

One step = the whole render of the configured frames (default 256 spp = 268,435,456 camera
paths) into a zeroed f32 accumulator resident in HBM, split across ranks by frame
(rank r renders frames k = r, r+N, ... — sample-interleaved), followed for
N > 1 by ONE RCCL sum-reduce of the W*H*3 accumulator to rank 0.  Strong scaling: the total
work is fixed as N grows.  The scene is packed by the product's Node host
(node/bin/pt-pack.js) before timing; scene upload is outside the timed region.

Prints ONE JSON line on rank 0 (contract in the task statement), with `roofline` for the
dominant kernel (the one with the most HIP-event time in the timed region, recorded by the
library around every launch on the render stream: pt_profile_enable/pt_profile_read).
Its algorithmic bytes per launch follow SURVEY.md §8d from the GPU's own work counters:
k_wf_trace (wavefront) moves 48 B per ray query (32 B ray read + 16 B hit write), so a launch
carries 48*Q / launches; the fused trace + shade kernel k_wf_step (the default on Cornell boxes)
carries 48*Q + 96*Q_ext (the path model without camera rays and accumulation) / launches; the
megakernel k_regen carries the whole path model B_alg = 48*Q + 96*Q_ext + 24 B per sample in
one launch.  `pipeline` gives B_alg over the
whole render.  `cpu_baseline` is the C oracle (oracle/pt_oracle.c) on the host cores, rank 0
at N=1 only.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

# before torch starts the HIP runtime: the dual-stream wavefront wants its two streams on
# hardware queues of their own, next to torch's and (N > 1) RCCL's streams; HIP's default is 4
# per process.  PT_BENCH_KEEP_QUEUES=1 keeps the inherited value (experiments).
if not os.environ.get("PT_BENCH_KEEP_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(8, int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)))

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "brown-cs2240-path-tracer_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 (vector), spec
L2_PEAK_GBS = 16800.0  # MI355X_MICROARCH.md: rows gathered from the XCDs' L2, 16.8-18.8 TB/s chip-wide


def pack_scene(scene: str, out_dir: str, W: int, H: int, spp: int, synthetic: int = 0, bvh: str = "reference",
               all_meshes: bool = False):
    """Pack with the product's Node host.  synthetic N: scripts/synth_scene.py's N-triangle
    Cornell-sized scene (the sweep of SURVEY.md §8(d)) instead of a reference scene."""
    if synthetic:
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import synth_scene  # noqa: E402
        xml = synth_scene.write(synthetic, os.path.join(out_dir, "synth"))
    else:
        xml = os.path.join(ROOT, "scenes", "scene_assets", scene + ".xml")
    extra = ["--bvh", bvh] + (["--native-bvh"] if synthetic or all_meshes else []) + (["--all-meshes"] if all_meshes else [])
    subprocess.run(["node", os.path.join(PKG, "node", "bin", "pt-pack.js"), xml, out_dir, "--width", str(W),
                    "--height", str(H), "--spp", str(spp), "--rr", "0.9", *extra], check=True)
    tri = np.fromfile(os.path.join(out_dir, "triangle_data.f32"), np.float32)
    bvh = np.fromfile(os.path.join(out_dir, "bvh_data.f32"), np.float32)
    meta = np.fromfile(os.path.join(out_dir, "meta.f32"), np.float32)
    return tri, bvh, meta


def cpu_baseline(tri, bvh, meta, depth, target_s=12.0):
    """C oracle on the host cores over a bounded sample of the same workload (~target_s of CPU work)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg only)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    W, H = int(meta[0]), int(meta[1])
    rows = max(1, H // 16)
    y0 = (H - rows) // 2
    t = time.perf_counter()
    oracle.render(tri, bvh, meta, 0, 1, 1, depth, y0=y0, y1=y0 + rows, nthreads=threads)
    per_frame = (time.perf_counter() - t) * H / rows  # one full frame
    if per_frame >= target_s:  # a band of central rows, one frame
        n_rows, nframes = max(8, int(H * target_s / per_frame)), 1
    else:  # whole frames
        n_rows, nframes = H, max(1, int(target_s / per_frame))
    y0 = (H - n_rows) // 2
    t = time.perf_counter()
    _, c = oracle.render(tri, bvh, meta, 0, nframes, 1, depth, y0=y0, y1=y0 + n_rows, nthreads=threads)
    dt = time.perf_counter() - t
    return {"value": round(c["samples"] / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/pt_oracle.c (CPU restatement of the reference WGSL; no CPU WebGPU adapter exists "
                      f"here) built gcc {oracle.lib_flags()} -fopenmp, {W}x{n_rows} rows x {nframes} frames of the "
                      f"same workload (depth {depth}), {threads} OpenMP threads, {c['samples']} samples in {dt:.2f} s"}


def load_traffic(kernel_prefix, scene: str, bvh: str, W: int, H: int, spp: int, depth: int, world: int,
                 field: str = "hbm_bytes_per_launch"):
    """Per-launch PMC figure of the render kernel (HBM bytes, or `valu_issue`) from the committed
    rocprofv3 passes (scripts/collect_traffic.sh -> profiles/traffic.json), when they match this
    configuration: (value, source) or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    key = f"{W}x{H}x{spp}x{depth}x{world}"
    entry = traffic_entry(t, scene, bvh, key) or {}
    cands = {k: v for k, v in entry.items() if k.startswith(kernel_prefix) and isinstance(v, dict) and field in v}
    # the timed instances: COUNT=false (template argument 4 of k_wf_step_bf<EXT, LDS, rcp, COUNT,
    # GEN> and of k_wf_trace<LDS, TRAV, COUNT, RING, PRUN> counted from 1 as 3; round 3's profiles name
    # a sixth k_wf_step_bf argument, the removed opt-in CULL, after COUNT); averaged per launch,
    # weighted by their dispatch counts when the summary has them (extension, shadow and the one
    # camera GEN launch per batch), else the plain mean of the instances (GEN left out)
    def timed_instance(name):
        args = [a.strip() for a in name[name.find("<") + 1:name.rfind(">")].split(",")]
        if name.startswith("k_wf_step_bf<"):
            return len(args) >= 4 and args[3] == "false" and (len(args) < 6 or args[4] == "false")
        if name.startswith("k_wf_trace<"):
            return len(args) >= 3 and args[2] == "false"
        return bool(args) and args[-1] == "false"

    def gen_instance(name):
        args = [a.strip() for a in name[name.find("<") + 1:name.rfind(">")].split(",")]
        return name.startswith("k_wf_step_bf<") and args[-1] == "true"

    timed = [k for k in cands if timed_instance(k)] or list(cands)
    if not timed:
        return None
    src = "profiles/traffic.json[" + key + "]: " + entry.get("_source", "rocprofv3 PMC passes (scripts/collect_traffic.sh)")
    wts = [cands[k].get("dispatches") for k in timed]
    if all(wts):
        return sum(cands[k][field] * w for k, w in zip(timed, wts)) / sum(wts), src
    timed = [k for k in timed if not gen_instance(k)] or timed  # no counts: leave GEN out
    return sum(cands[k][field] for k in timed) / len(timed), src


def gpu_sysfs_dir(pci_bus_id: str | None):
    """The amdgpu sysfs directory of the GPU at this PCI address (torch's device properties give
    domain:bus:device); None when not found (no sysfs, another driver)."""
    import glob
    found = []
    for c in sorted(glob.glob("/sys/class/drm/card*/device")):
        try:
            addr = os.path.basename(os.path.realpath(c))
        except OSError:
            continue
        if os.path.exists(os.path.join(c, "pp_dpm_sclk")) and addr not in [a for a, _ in found]:
            found.append((addr, c))
    if pci_bus_id:
        for addr, c in found:
            if addr.lower().startswith(pci_bus_id.lower()):
                return c
    return found[0][1] if len(found) == 1 else None


def gpu_state(dev_dir: str | None) -> dict | None:
    """The GPU's clock and power state from sysfs (read-only files; nothing is set): the current DPM
    level of each clock domain (pp_dpm_*: the line marked '*'), the hwmon sclk, power (average or
    input) and cap, and temperatures.  Lets a bench line from one box be compared with another's
    (a 5 % spread between boxes with nothing recorded to tell a slow box from a slow
    build)."""
    if not dev_dir:
        return None
    import glob
    out = {}

    def rd(path):
        try:
            with open(path) as f:
                return f.read()
        except OSError:
            return None
    for dom in ("sclk", "mclk", "fclk", "socclk"):
        txt = rd(os.path.join(dev_dir, f"pp_dpm_{dom}"))
        if not txt:
            continue
        for line in txt.splitlines():
            if line.rstrip().endswith("*"):
                v = line.split(":", 1)[-1].replace("*", "").strip().lower()
                try:
                    out[f"{dom}_mhz"] = float(v.replace("mhz", "").strip())
                except ValueError:
                    out[f"{dom}_level"] = v
    for hw in sorted(glob.glob(os.path.join(dev_dir, "hwmon", "hwmon*")))[:1]:
        for name, key, scale in (("freq1_input", "sclk_hwmon_mhz", 1e-6), ("power1_average", "power_w", 1e-6),
                                 ("power1_input", "power_input_w", 1e-6), ("power1_cap", "power_cap_w", 1e-6),
                                 ("temp1_input", "temp_edge_c", 1e-3), ("temp2_input", "temp_junction_c", 1e-3),
                                 ("temp3_input", "temp_mem_c", 1e-3)):
            v = rd(os.path.join(hw, name))
            if v is not None:
                try:
                    out[key] = round(float(v.strip()) * scale, 1)
                except ValueError:
                    pass
    perf = rd(os.path.join(dev_dir, "power_dpm_force_performance_level"))
    if perf:
        out["perf_level"] = perf.strip()
    return out or None


class GpuStateSampler:
    """Samples gpu_state every `period` s on a host thread while the timed region runs (sysfs reads
    only); summary() gives min / median / max of the numeric fields."""

    def __init__(self, dev_dir, period=0.05):
        import threading
        self.dev_dir, self.period, self.samples = dev_dir, period, []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True) if dev_dir else None

    def _run(self):
        while not self._stop.is_set():
            st = gpu_state(self.dev_dir)
            if st:
                self.samples.append(st)
            self._stop.wait(self.period)

    def __enter__(self):
        if self._t:
            self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._t:
            self._t.join()

    def summary(self):
        if not self.samples:
            return None
        keys = sorted({k for s in self.samples for k, v in s.items() if isinstance(v, float)})
        return {"samples": len(self.samples),
                **{k: [min(v), float(np.median(v)), max(v)] for k in keys
                   for v in [[s[k] for s in self.samples if k in s]]}}


def traffic_entry(t: dict, scene: str, bvh: str, key: str):
    """profiles/traffic.json's entry for this workload: the scene- and tree-qualified key (written by
    scripts/summarize_traffic.py since round 6), else the plain size key when its source names the
    same scene (older entries; reference trees only)."""
    q = t.get(f"{scene}|{bvh}|{key}")
    if q is not None:
        return q
    e = t.get(key)
    if e and bvh == "reference" and f"({scene}.xml " in e.get("_source", ""):
        return e
    return None


def load_valu_exec(scene: str, bvh: str, W: int, H: int, spp: int, depth: int, world: int, weights: dict):
    """The VALU work the step's kernels actually execute, from the committed PMC pass
    (scripts/collect_traffic.sh -> profiles/traffic.json, this configuration's key): per kernel family
    (k_wf_step, k_wf_trace, k_wf_leafpass, ...; instances summed by their dispatches) the
    FMA-calibrated issue density k x SQ_ACTIVE_INST_VALU / (128 x GRBM_GUI_ACTIVE) times the lane use
    SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU) = the fraction of the SIMDs' f32 lane-op peak
    the kernel executes; the step's figure weights each family by its time in the warm-up step
    (`weights`: family -> ms).  Unlike valu_alg (the reference's work at this rate) it counts what the
    kernels do, so it stays below 1.  None without a matching PMC pass."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    key = f"{W}x{H}x{spp}x{depth}x{world}"
    try:
        with open(path) as f:
            t = traffic_entry(json.load(f), scene, bvh, key)
        with open(os.path.join(ROOT, "profiles", "valu_calibration.json")) as f:
            k_cal = json.load(f)["k_active"]
    except (OSError, ValueError, KeyError):
        return None
    if not t:
        return None

    def family(name):  # the bench's kernel names (pt_profile_read); None for the counted render's instances
        f = name.split("<")[0]
        args = [a.strip() for a in name[name.find("<") + 1:name.rfind(">")].split(",")] if "<" in name else []
        counted = {"k_wf_step_bf": 3, "k_wf_trace": 2, "k_wf_trace_pre": 2, "k_wf_shade": 1, "k_wf_generate": 0}
        if f in counted and len(args) > counted[f] and args[counted[f]] == "true":
            return None
        if f == "k_wf_shade":
            return "k_wf_shade_ext" if args and args[0] == "true" else "k_wf_shade_shadow"
        return {"k_wf_step_bf": "k_wf_step", "k_wf_trace_pre": "k_wf_trace"}.get(f, f)
    fam = {}
    for name, e in t.items():
        v = e.get("valu_counters") if isinstance(e, dict) else None
        if not v or not v.get("GRBM_GUI_ACTIVE") or not v.get("SQ_ACTIVE_INST_VALU"):
            continue
        f = family(name)
        if f is None:
            continue
        n = e.get("dispatches") or 1
        a = fam.setdefault(f, [0.0, 0.0, 0.0])
        a[0] += v["SQ_ACTIVE_INST_VALU"] * n
        a[1] += v.get("SQ_THREAD_CYCLES_VALU", 0.0) * n
        a[2] += v["GRBM_GUI_ACTIVE"] * n
    per = {}
    for f, (act, thr, grbm) in fam.items():
        dens, lane = k_cal * act / (128.0 * grbm), thr / (64.0 * act)
        per[f] = {"issue_density": round(dens, 4), "lane_use": round(lane, 4), "frac": round(dens * lane, 4),
                  "step_ms_warmup": round(weights.get(f, 0.0), 3)}
    per = {f: p for f, p in per.items() if p["step_ms_warmup"] > 0}  # the step's own kernels
    wsum = sum(p["step_ms_warmup"] for p in per.values())
    if not per or wsum <= 0:
        return None
    return {"frac": round(sum(p["frac"] * p["step_ms_warmup"] for p in per.values()) / wsum, 4), "kernels": per,
            "def": "per kernel: (k x SQ_ACTIVE_INST_VALU / (128 x GRBM_GUI_ACTIVE)) x (SQ_THREAD_CYCLES_VALU / (64 x "
                   "SQ_ACTIVE_INST_VALU)), the executed fraction of the f32 lane-op peak; the step: weighted by each "
                   "kernel's time in the warm-up step",
            "source": f"profiles/traffic.json[{scene}|{bvh}|{key}] (scripts/collect_traffic.sh) "
                      "+ profiles/valu_calibration.json"}


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: run this same command as N ranks
    under torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) and return its exit
    code.  The parent has not touched the GPU (torch is not even imported yet): the ranks are
    fresh child processes, so no process that initialised HIP is replaced."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def traffic_note(kernel_prefix, scene: str, bvh: str, W: int, H: int, spp: int, depth: int, world: int, field: str):
    """A text field of the render kernel's entry in profiles/traffic.json (e.g. the VALU calibration)."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            t = traffic_entry(json.load(f), scene, bvh, f"{W}x{H}x{spp}x{depth}x{world}") or {}
    except (OSError, ValueError):
        return None
    for k, v in t.items():
        if k.startswith(kernel_prefix) and isinstance(v, dict) and field in v:
            return v[field]
    return None


def load_trace_union(W: int, H: int, spp: int, depth: int, world: int):
    """The rocprofv3 kernel-trace busy time of the render kernel for this configuration
    (scripts/trace_union.py -> profiles/trace_union.json), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "trace_union.json")) as f:
            return json.load(f).get(f"{W}x{H}x{spp}x{depth}x{world}")
    except (OSError, ValueError):
        return None


def metric_name(scene: str, W: int, H: int, depth: int) -> str:
    """BASELINE.json's metric, for the workload actually run (its headline is CornellBox 1024^2 depth 8)."""
    return f"Msamples/s (paths/s) {scene} {W}x{H} depth {depth}"


def native_multi(args):
    """bench.py --native-multi --gpus N: ONE process renders the step over N devices with the C ABI's
    pt_render_multi (frames dealt round-robin, one host thread per device, one ncclReduce onto
    device 0 inside the library).  Host-buffer call: the accumulator upload and read-back (12 MB
    each way at 1024^2) over PCIe are inside the timed step."""
    import pt_amd
    n = max(1, args.gpus)
    if args.synthetic:
        args.scene = f"synthetic-{args.synthetic}"
    with tempfile.TemporaryDirectory() as td:
        tri, bvh, meta = pack_scene(args.scene, td, args.width, args.height, args.spp, args.synthetic, args.bvh,
                                    args.all_meshes)
    W, H = int(meta[0]), int(meta[1])
    mode = {"auto": pt_amd.MODE_AUTO, "megakernel": pt_amd.MODE_MEGAKERNEL, "wavefront": pt_amd.MODE_WAVEFRONT}[args.mode]
    if args.reduce:
        pt_amd.set_option("reduce", args.reduce)
    scenes = [pt_amd.Scene(tri, bvh, device=g) for g in range(n)]
    acc = np.zeros((H, W, 3), np.float32)
    for _ in range(args.warmup):
        acc[:] = 0
        pt_amd.render_multi(scenes, meta, 0, args.spp, 1, args.depth, mode, accum=acc)
    t = []
    for _ in range(args.steps):
        acc[:] = 0
        t0 = time.perf_counter()
        pt_amd.render_multi(scenes, meta, 0, args.spp, 1, args.depth, mode, accum=acc)
        t.append(time.perf_counter() - t0)
    for s in scenes:
        s.close()
    elapsed = float(np.sum(t))
    total = W * H * args.spp
    out = {"metric": metric_name(args.scene, W, H, args.depth), "value": round(total / (elapsed / args.steps) / 1e6, 3),
           "unit": "Msamples/s", "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "f32",
           "data": f"synthetic (reference {args.scene}.xml scene packed by the Node host; RNG salts t_k = k)",
           "config": {"workload": f"{args.scene}.xml {W}x{H} {args.spp}spp depth {args.depth}, rr 0.9, frames dealt "
                                  f"round-robin over {n} devices in one process (pt_render_multi), host accumulator "
                                  f"(PCIe upload + read-back in the step)",
                      "mode": args.mode, "samples_per_step": total,
                      "reduce": (args.reduce or "rccl") if n > 1 else
                      ("rccl (one-rank communicator)" if args.reduce == "rccl" else "none")}}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 10 timed steps (~1 s at configs[1]): the first step's ramp and the last step's per-launch events
    # weigh half what they did over 5 (r06y2: 2,866 over 10 steps against 2,848 over 5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene", default="CornellBox")
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--mode", default="auto", choices=["auto", "megakernel", "wavefront"])
    ap.add_argument("--synthetic", type=int, default=0, help="N-triangle synthetic Cornell-sized scene (BVH sweep)")
    ap.add_argument("--bvh", default="reference", choices=["reference", "sah"], help="sah: the fast (non-parity) tree")
    ap.add_argument("--all-meshes", action="store_true", help="every primitive of the scene (reference: first only)")
    ap.add_argument("--native-multi", action="store_true",
                    help="one process drives --gpus devices through pt_render_multi (RCCL reduce inside the library)")
    ap.add_argument("--reduce", choices=["rccl", "ordered"], help="--native-multi: pt_render_multi's reduction")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true", help="diagnostic: no per-launch HIP events")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="library option (pt_set_option) for A/B and profiling runs; repeatable")
    ap.add_argument("--readback", choices=["pt", "torch"], default="pt",
                    help="the step's accumulator-to-host copy: pt_readback_async (16 blocks) or torch's copy_")
    ap.add_argument("--share-of", type=int, default=0, metavar="N",
                    help="one GPU renders exactly rank --share-rank's frames of an N-rank run (frames r, r+N, ...; no "
                         "reduce): the per-rank share whose time bounds N-GPU strong scaling (DESIGN.md section 7)")
    ap.add_argument("--share-rank", type=int, default=0)
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the rank plumbing (launch, sharding, reduce, timing, JSON line); renders "
                         "nothing and reports no value")
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None and not args.native_multi:
        sys.exit(launch_ranks(args.gpus))  # N ranks of this command; nothing here touched the GPU
    world = int(world_env or "1")
    if args.gpus > 1 and world != args.gpus and not args.native_multi:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: n_gpus must be the ranks that render")

    import torch
    import torch.distributed as dist

    from pt_amd.shard import frames_for_rank, reduce_accum

    if args.native_multi:
        if world != 1:
            raise SystemExit("--native-multi is single-process (it drives --gpus devices itself)")
        return native_multi(args)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # PT_BENCH_BACKEND=gloo: rehearsal of the N > 1 path with several ranks on fewer GPUs (the
    # reduce then goes through host memory); the driver's runs use RCCL, one rank per GPU
    backend = os.environ.get("PT_BENCH_BACKEND", "gloo" if args.dry_run else "nccl")
    if world > 1:
        dist.init_process_group(backend)
    ranks_seen = dist.get_world_size() if world > 1 else 1
    if args.dry_run:
        return dry_run(args, rank, world, ranks_seen, backend, dist, frames_for_rank, reduce_accum)
    import pt_amd
    for kv in args.opt:
        k, _, v = kv.partition("=")
        pt_amd.set_option(k, v)
    if backend == "gloo":
        local_rank %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    if args.synthetic:
        args.scene = f"synthetic-{args.synthetic}"
    with tempfile.TemporaryDirectory() as td:
        tri, bvh, meta = pack_scene(args.scene, td, args.width, args.height, args.spp, args.synthetic, args.bvh,
                                    args.all_meshes)
    W, H = int(meta[0]), int(meta[1])
    mode = {"auto": pt_amd.MODE_AUTO, "megakernel": pt_amd.MODE_MEGAKERNEL, "wavefront": pt_amd.MODE_WAVEFRONT}[args.mode]
    scene = pt_amd.Scene(tri, bvh, device=local_rank)
    # frames of this rank: k = rank, rank + world, ... (pt_amd/shard.py)
    frame0, nframes, fstride = frames_for_rank(rank, world, args.spp)
    if args.share_of > 1:  # one rank's share of an N-rank run, rendered alone
        if world != 1:
            raise SystemExit("--share-of times one rank's share on one GPU (no launcher)")
        frame0, nframes, fstride = frames_for_rank(args.share_rank, args.share_of, args.spp)
    try:
        props = torch.cuda.get_device_properties(dev)
        pci = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
    except Exception:  # noqa: BLE001  (older torch: no PCI fields)
        pci = None
    sysfs = gpu_sysfs_dir(pci)
    state_start = gpu_state(sysfs)
    stream = torch.cuda.Stream(device=dev)
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device=dev)
    # the step ends with the accumulator on the host ("from the first kernel launch to
    # the accumulator on the host"; the reference copies it to a MAP_READ buffer each frame,
    # program-raymarch.ts:262-293): rank 0 copies the reduced accumulator to pinned host memory.
    # Two accumulators: step k renders into slot k % 2 while a copy stream brings step k - 1's to the
    # host (readback pipelined with the next step's render, ~0.23 ms of PCIe per 12 MB at 1024^2 —
    # 2 % of a rank's share of an 8-GPU run, profiles/r05o_share.log); every step's copy completes
    # inside the timed region, which ends with both streams drained.
    accs = [acc, torch.zeros_like(acc)]
    hosts = ([torch.empty((H, W, 3), dtype=torch.float32, pin_memory=True) for _ in range(2)] if rank == 0
             else [None, None])
    copy_stream = torch.cuda.Stream(device=dev)
    slot_free = [None, None]  # per slot: the event after which its accumulator may be zeroed again
    nstep = [0]

    def step(ev0=None, ev1=None):
        k = nstep[0] % 2
        nstep[0] += 1
        a = accs[k]
        with torch.cuda.stream(stream):
            if slot_free[k] is not None:
                stream.wait_event(slot_free[k])  # step k - 2's host copy of this slot is done
            a.zero_()
            if ev0 is not None:
                ev0.record(stream)
            scene.render_async(meta, frame0, nframes, fstride, args.depth, mode, a.data_ptr(), stream.cuda_stream)
            if ev1 is not None:
                ev1.record(stream)
            reduce_accum(a, dist)
            done = torch.cuda.Event()
            done.record(stream)
        if hosts[k] is not None:
            with torch.cuda.stream(copy_stream):
                copy_stream.wait_event(done)
                if args.readback == "pt":  # pt_readback_async: a 16-block copy kernel
                    scene.readback_async(a.data_ptr(), a.numel(), hosts[k].data_ptr(), copy_stream.cuda_stream)
                else:  # the runtime's copy (a blit kernel of ~512 blocks on this stack)
                    hosts[k].copy_(a, non_blocking=True)
                done = torch.cuda.Event()
                done.record(copy_stream)
        slot_free[k] = done

    def drain():
        stream.synchronize()
        copy_stream.synchronize()

    # work counters for the roofline's algorithmic bytes (separate pass, not timed)
    cnt = torch.zeros(6, dtype=torch.int64, device=dev)
    with torch.cuda.stream(stream):
        tmp = torch.zeros_like(acc)
        scene.render_async(meta, frame0, nframes, fstride, args.depth, mode, tmp.data_ptr(), stream.cuda_stream,
                           d_counters_ptr=cnt.data_ptr())
    stream.synchronize()
    c = cnt.cpu().tolist()
    samples_c, q_ext, q_sh = c[0], c[1], c[2]
    del tmp

    # warm-up with every kernel timed: it names the dominant kernel, the only one whose launches
    # carry events in the timed region (events around every launch cost ~5 % of the step)
    scene.profile_enable(True)
    for _ in range(args.warmup):
        step()
    drain()
    prof_warm = scene.profile_read()
    scene.profile_enable(False)
    dominant = max(prof_warm, key=lambda k: prof_warm[k]["total_ms"]) if prof_warm else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # one event pair per step, read after the loop: the host enqueues step k + 1 while the GPU still
    # runs step k (a synchronisation per step would leave the GPU idle while ~150 launches are issued)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    # the dominant kernel's launches carry HIP events in the LAST timed step only: an event pair per
    # launch costs the step ~1 % at configs[1] (144 launches in 95 ms) and ~5 % for one rank's
    # 1/8 share (36 launches in 13 ms; profiles/r05ae_share_events.jsonl), so the other steps run
    # uninstrumented and the kernel's average launch and busy time come from that one step
    scene.profile_select(dominant)
    timed = not args.no_kernel_timing and dominant is not None
    with GpuStateSampler(sysfs) as sampler:
        t0 = time.perf_counter()
        for i, (ev0, ev1) in enumerate(evs):
            if timed and i == len(evs) - 1:
                scene.profile_enable(True)
            step(ev0, ev1)
        drain()
        render_ms = [ev0.elapsed_time(ev1) for ev0, ev1 in evs]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    state_end = gpu_state(sysfs)
    prof = scene.profile_read()
    scene.profile_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend != "gloo" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    scene.check()  # a device-side failure of any timed render (pt_scene_check) fails the bench
    total_samples = W * H * (nframes if args.share_of > 1 else args.spp)
    ms_per_step = elapsed / args.steps * 1e3
    value = total_samples / (elapsed / args.steps) / 1e6
    r_ms = float(np.mean(render_ms))
    b_alg = (48.0 * (q_ext + q_sh) + 96.0 * q_ext + 24.0 * samples_c)  # bytes per render
    if prof:
        kernel = max(prof, key=lambda k: prof[k]["total_ms"])
        launches_per_render = prof[kernel]["launches"]  # of the last timed step
        k_ms = prof[kernel]["avg_ms"]
        busy_ms = prof[kernel]["busy_ms"]  # union of the launches' intervals in that step
        if kernel in ("k_wf_trace", "k_wf_leafpass"):
            # the traversal's model: a ray record read and a hit record written per query (the big-leaf
            # pass reads the same records and writes a key per query that meets a big leaf's boxes)
            bytes_per_launch = 48.0 * (q_ext + q_sh) / launches_per_render
        elif kernel == "k_wf_step":  # fused trace + shade: the path model minus camera rays and accumulation
            bytes_per_launch = (48.0 * (q_ext + q_sh) + 96.0 * q_ext) / launches_per_render
        else:  # the megakernel: the whole path model in one launch
            bytes_per_launch = b_alg / launches_per_render
        # achieved = the algorithmic bytes of all of a step's launches over the time the kernel
        # is busy in that step (launches of the batch's parts overlap on their streams, so the
        # per-launch event time over-counts: it is reported, not used)
        achieved = bytes_per_launch * launches_per_render / (busy_ms * 1e-3) / 1e9
    else:  # --no-kernel-timing (diagnostic)
        kernel, launches_per_render, k_ms, busy_ms, bytes_per_launch, achieved = "n/a", 0, 0.0, 0.0, 0.0, 0.0
    pipeline = b_alg / (r_ms * 1e-3) / 1e9
    # SURVEY.md §8d's secondary figure, the algorithmic VALU work, from the same counters (the
    # reference's own units: every triangle test and node step its traversal makes, and the path
    # logic per bounce): 40 flop per triangle test + 2 x 24 per node step + 150 per extension query
    flop_per_render = 40.0 * c[4] + 48.0 * c[3] + 150.0 * q_ext
    valu_tflops = flop_per_render / max(samples_c, 1) * value * 1e6 / 1e12  # at the step's samples/s
    # and the scene bytes the reference's traversal reads (SURVEY.md §8d secondary: 56 B per node
    # step, 52 B per triangle test, 60 B per material fetch — one per extension query), the figure
    # that bounds the traversal scenes from L2 rather than HBM
    scene_per_render = 56.0 * c[3] + 52.0 * c[4] + 60.0 * q_ext
    scene_gbs = scene_per_render / max(samples_c, 1) * value * 1e6 / 1e9

    if rank == 0:
        prefixes = {"k_wf_trace": ("k_wf_trace<", "k_wf_trace_bf<"), "k_wf_step": ("k_wf_step_bf<",),
                    "k_wf_leafpass": ("k_wf_leafpass<",)}
        pre = prefixes.get(kernel, (kernel + "<",))
        # the committed PMC / trace figures describe the full configuration (not a rank's share)
        full = args.share_of <= 1
        traffic = load_traffic(pre, args.scene, args.bvh, W, H, args.spp, args.depth, world) if full else None
        valu = (load_traffic(pre, args.scene, args.bvh, W, H, args.spp, args.depth, world, field="valu_issue")
                if full else None)
        valu_cal = traffic_note(pre, args.scene, args.bvh, W, H, args.spp, args.depth, world, "valu_issue_calibration")
        tu = load_trace_union(W, H, args.spp, args.depth, world) if full else None
        if tu and tu.get("kernel") != kernel:
            tu = None
        out = {
            "metric": metric_name(args.scene, W, H, args.depth),
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"synthetic ({args.synthetic} triangles in the Cornell box, scripts/synth_scene.py, seed 1234; "
                     if args.synthetic else f"synthetic (reference {args.scene}.xml scene ") +
                    f"packed by the Node host, {args.bvh} BVH" + (", all meshes" if args.all_meshes else "") +
                    "; RNG salts t_k = k)",
            "config": {"workload": f"{args.scene}.xml {W}x{H} {args.spp}spp depth {args.depth}, rr 0.9, "
                                   f"frames sharded k mod {world}" + ((", RCCL sum-reduce of the f32 accumulator" if backend == "nccl" else
                                                                         f", {backend} sum-reduce through host memory (rehearsal)")
                                                                        if world > 1 else ""),
                       "mode": args.mode, "bvh": args.bvh, "samples_per_step": total_samples,
                       "timed_to": "accumulator on the host (rank 0: pinned device-to-host copy after the "
                                   "reduce, every step's inside the timed region; step k's copy overlaps step "
                                   "k + 1's render, two accumulators)",
                       "readback": ("pt_readback_async (16-block copy kernel)" if args.readback == "pt"
                                    else "torch copy_ (runtime blit)"),
                       "ranks": ranks_seen, "backend": backend if world > 1 else None,
                       "options": dict(kv.partition("=")[::2] for kv in args.opt) or None,
                       "scene_triangles": int((int(tri[4]) - int(tri[3])) // 4), "bvh_floats": int(bvh.size),
                       "share": ({"of": args.share_of, "rank": args.share_rank, "frames": nframes, "stride": fstride,
                                  "implied_aggregate_before_reduce": round(value * args.share_of, 3)}
                                 if args.share_of > 1 else None)},
            # the GPU's clocks, power and temperatures (sysfs, read-only) before the warm-up, sampled
            # every 50 ms through the timed region (min / median / max), and after it
            "gpu_state": {"pci": pci, "sysfs": sysfs, "start": state_start, "timed": sampler.summary(),
                          "end": state_end},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic[0] * launches_per_render / (busy_ms * 1e-3) / 1e9 if traffic and busy_ms else None,
                         "traffic_unit": "GB/s (PMC HBM bytes per launch x launches / busy time)",
                         "traffic_bytes_per_launch": round(traffic[0]) if traffic else None,
                         "traffic_source": traffic[1] if traffic else None,
                         "kernel": kernel, "kernel_avg_ms": round(k_ms, 4),
                         "kernel_busy_ms_per_step": round(busy_ms, 3),
                         "rocprof_busy_ms_per_step": tu["busy_ms_per_step_rocprof"] if tu else None,
                         "rocprof_achieved": (round(bytes_per_launch * launches_per_render /
                                                    (tu["busy_ms_per_step_rocprof"] * 1e-3) / 1e9, 2) if tu else None),
                         "rocprof_source": ("profiles/trace_union.json: union of the kernel's dispatch intervals in a "
                                            "rocprofv3 --kernel-trace of bench.py (scripts/trace_union.py, " +
                                            tu["source"] + ")") if tu else None,
                         "achieved_def": "algorithmic bytes per launch (SURVEY.md 8d model from the GPU's work counters) x "
                                         "launches per step / the kernel's busy time per step (union of its launches' "
                                         "HIP-event intervals on every part stream, in the last timed step: the "
                                         "others carry no events)",
                         "launches_per_step": launches_per_render, "bytes_per_launch": round(bytes_per_launch),
                         "queries_per_sample": round((q_ext + q_sh) / max(samples_c, 1), 3),
                         "valu_alg_frac": round(valu_tflops / VALU_PEAK_TFLOPS, 4),
                         "valu_alg": {"flop_per_sample": round(flop_per_render / max(samples_c, 1), 1),
                                      "achieved": round(valu_tflops, 2), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                                      "frac": round(valu_tflops / VALU_PEAK_TFLOPS, 4),
                                      "def": "(40 x triangle tests + 48 x node steps + 150 x extension queries) of "
                                             "the reference's traversal, from the GPU's work counters (SURVEY.md 8d "
                                             "secondary), per sample x samples/s of the step / the f32 vector peak"},
                         "scene_bytes": {"bytes_per_sample": round(scene_per_render / max(samples_c, 1), 1),
                                         "achieved": round(scene_gbs, 1), "peak": L2_PEAK_GBS, "unit": "GB/s",
                                         "vs_l2": round(scene_gbs / L2_PEAK_GBS, 4),
                                         "def": "(56 x node steps + 52 x triangle tests + 60 x extension queries) "
                                                "bytes of the reference's traversal, from the GPU's work counters "
                                                "(SURVEY.md 8d secondary), per sample x samples/s, against the chip's "
                                                "L2 gather rate (MI355X_MICROARCH.md: 16.8-18.8 TB/s, the lower end); "
                                                "above 1 where the kernels do not read what that traversal would "
                                                "(scenes brute-forced from LDS, leaf entries culled by chunks)"},
                         "pipeline": {"bytes_per_sample": round(b_alg / max(samples_c, 1), 1),
                                      "achieved": round(pipeline, 2), "frac": round(pipeline / HBM_PEAK_GBS, 4)},
                         # not a utilisation (it can exceed 1): VALU wave-instructions priced at the
                         # SIMD cycles of a chain of v_fma_f32, over all SIMD cycles
                         "valu_fma_equiv_density": ({"value": round(valu[0], 4),
                                                     "def": "k x SQ_ACTIVE_INST_VALU / (128 x GRBM_GUI_ACTIVE), kernel "
                                                            "alone (PMC pass), k = the SIMD cycles per v_fma_f32 "
                                                            "wave-instruction at peak (pt_selftest_valu reads 1.0); "
                                                            "an FMA-equivalent issue density, above 1 when the mix "
                                                            "issues faster than FMA chains",
                                                     "calibration": valu_cal or "uncalibrated (k = 4)",
                                                     "source": valu[1]} if valu else None),
                         "kernels_ms_warmup_step": {k: round(v["total_ms"] / max(args.warmup, 1), 3)
                                                    for k, v in prof_warm.items()},
                         "valu_exec": (load_valu_exec(args.scene, args.bvh, W, H, args.spp, args.depth, world,
                                                      {k: v["total_ms"] / max(args.warmup, 1) for k, v in prof_warm.items()})
                                       if full else None),
                         "render_ms_steps": [round(x, 2) for x in render_ms]},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(tri, bvh, meta, args.depth)
        print(json.dumps(out), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()


def dry_run(args, rank, world, ranks_seen, backend, dist, frames_for_rank, reduce_accum):
    """--dry-run: the N > 1 plumbing without a GPU (CPU tests): each rank takes its frame share,
    a CPU accumulator holding its frame count goes through the same reduce, the step is timed
    with the same barrier + max-over-ranks, and rank 0 prints the line (value null)."""
    import torch
    W, H = args.width, args.height
    frame0, nframes, fstride = frames_for_rank(rank, world, args.spp)
    acc = torch.zeros((H, W, 3), dtype=torch.float32)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        acc.fill_(float(nframes))
        reduce_accum(acc, dist)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        frames_total = float(acc[0, 0, 0])  # the reduce summed every rank's frame count
        print(json.dumps({"metric": metric_name(args.scene, W, H, args.depth), "value": None, "unit": "Msamples/s",
                          "n_gpus": ranks_seen, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "dry run (no render)",
                          "dry_run": True, "config": {"ranks": ranks_seen, "backend": backend if world > 1 else None,
                                                      "frames_reduced": frames_total}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
