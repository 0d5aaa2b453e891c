"""
Benchmark: aligned records/s for cell + gene metrics on MI355X (BASELINE.json).

One step = one pass of the hot path over this rank's synthetic shard, already
resident in HBM: per-cell metrics (RUN mode over the cell-sorted records) plus
per-gene metrics (grouped per-gene partials, an RCCL all-reduce across ranks
when N > 1, finalize), with both sets of entity rows copied back to the host.

Workload: 100M cell-sorted records over 10k cells
(lognormal(0,1) reads per cell), 30k genes (Zipf 1.1, plus None and multi-gene
ids), 10-mer UMIs; generated on the GPU.

* N = 1: config 2 (the default).
* N > 1: config 3 by default (BASELINE.json: "Same 100M-read workload ... across
  2/4/8 GPUs"): every rank generates the SAME 100M-record set and keeps its
  SplitBam-style shard -- a contiguous cell range balanced by record count
  (distributed.shard_bounds) -- so N GPUs split one 100M-record job: strong
  scaling, value = 100M x steps / max-over-ranks time.  `--config 2` at N > 1
  gives each rank its own 100M records of disjoint cells instead (weak scaling).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
       (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
Rank 0 prints ONE JSON line.
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_HBM = 8.0e12  # MI355X HBM3E spec, MI355X_MICROARCH.md
PROFILE_STEPS = 2  # untimed steps with every kernel timed (the per-kernel table)

# The unmodified reference Python gatherer timed in the build container (BASELINE.md "Measured CPU
# reference"; it cannot run on the GPU box): context for `value`, not the cpu_baseline leg.
REFERENCE_PYTHON = {
    "value": 39038.0,
    "unit": "records/s",
    "cores": 1,
    "kind": "reference (Python, unmodified)",
    "host": "build container: Intel Xeon, 8 cores, 1 thread per core (not the GPU box)",
    "sample": "GatherCellMetrics aggregation of 200k pre-decoded 10x-v2-shaped records, 20 cells, 30k genes; "
              "stub pysam records, BAM decode excluded (BASELINE.md table, SURVEY.md 6)",
    "value_8_processes": 268000.0,
}

# Algorithmic HBM bytes per record per launch of each kernel.
ALG_BYTES = {
    "hash_tile": 20,         # read payload w0 + w1 (16) + bucket descriptor (2), write dflags (2)
    "bucket_scatter": 32,    # read payload 16, write payload 16 (records of the level's segments)
    "bucket_hist": 8,        # read w0
    "build_keys": 48,        # read cell/gene/umi/ref/pos (20) + bits/xf (2) + uy/gq/cy (10), write payload (16)
    "big_bucket": 18,        # read payload w0 + w1 (16) of the big buckets' records, write dflags (2)
    "gene_emit": 24,         # read gene/bits/xf/dflags/uy/gq (16), write the 8-byte gene payload (16 when wide)
    "gene_reduce": 8,        # read the 8-byte gene payload (16 when wide)
    "tag_row_scatter": 68,   # config 5, per pass: read a 32-byte row (SoA or packed), write it (+ 4-byte key)
    "tag_row_hist": 4,       # config 5, per pass: read the cell key
    "tag_pack": 64,          # tag sort with a tiebreak: read the 32-byte SoA record, write it packed
    "tag_keys": 28,          # read the packed record's key words (16), write key 8 + index 4
    "tag_pack_keys": 80,     # read the SoA record (32) + tiebreak (4), write the packed row (32) + key 8 + index 4
    "radix_onesweep": 24,    # (opt-in onesweep) read key 8 + value 4, write key 8 + value 4
    "radix_hist_all": 8,
    "tag_unpack": 64,        # gather the packed record (32), write the SoA columns (32)
    # config 5's sort (round 6): the 32-bit group keys (tagsort.h); the 64-bit general path's passes
    # move 24 and 8 bytes instead, and the bench does not run them
    "radix_downsweep": 16,   # read key 4 + value 4, write key 4 + value 4
    "radix_upsweep": 4,      # read key 4
    "tag_group_keys": 72,    # read the SoA record (32) + tiebreak (4), write the row (32) + group key (4)
    "tag_group_hist": 8,     # read the cell and umi columns (the MSD digit of the group key)
    "tag_group_msd": 72,     # the MSD pass: read the SoA record (32) + tiebreak (4), write the row (32) + key (4)
    "tag_group_wave": 72,    # read the group key (4) + the permutation (4), gather the row (32), write SoA (32)
    "tag_group_long": 72,    # the same for the records of groups longer than a wave
    "reduce_sorted": 12,
    "heads": 4,              # read the entity column
    "welford": 10,
}


# HIP-event kernel names (engine profile) -> rocprofv3 kernel names (tools/pmc_traffic.py keys)
# engine profile names -> the kernels (rocprofv3 names, sct::k_*) launched under them; a name
# covering several kernels gets their dispatch-weighted mean bytes per launch
PMC_NAMES = {"build_keys": ["build_keys_run"], "heads": ["heads4", "heads"], "fill": ["fill_spans"],
             "scan": ["scan_wide", "scan_reduce", "scan_small", "scan_apply"],
             "tag_pack": ["pack"], "tag_keys": ["field_keys", "round_keys"], "tag_ties": ["tie_wave", "tie_wave2"],
             "tag_pack_keys": ["pack_field_keys"],
             "tag_long_keys": ["long_keys"], "tag_long_scatter": ["long_scatter"], "tag_unpack": ["unpack"],
             "tag_row_hist": ["row_hist"], "tag_row_scatter": ["row_scatter"],
             "tag_group_keys": ["pack_group_keys"], "tag_group_wave": ["group_wave"],
             "tag_group_long": ["group_long"], "tag_group_iota": ["iota"], "tag_group_hist": ["gmsd_hist"],
             "tag_group_msd": ["gmsd_scatter"], "tag_group_plan": ["gseg_plan"],
             "radix_upsweep": ["radix_upsweep", "gseg_upsweep"], "radix_downsweep": ["radix_downsweep", "gseg_downsweep"]}


def pmc_bytes_per_launch(d, name):
    """HBM bytes per launch of profile name `name` from a pmc_traffic.json, or None."""
    ks = [k for k in PMC_NAMES.get(name, [name]) if k in d.get("kernels", {})]
    if not ks:
        return None
    w = [max(1, d["kernels"][k].get("dispatches", 1)) for k in ks]
    return sum(d["kernels"][k]["hbm_bytes_per_launch"] * x for k, x in zip(ks, w)) / sum(w)


def pipeline_bytes(args, dims):
    """B_alg = 32 + 12 + 24 P + 44 bytes/record, P = ceil(b / 8) LSD passes with
    b = bits(cells per shard) + bits(gene ids) + bits(umi ids) -- a property of the workload."""
    def bits(v):
        return max(0, int(v - 1).bit_length())
    b = bits(args.cells) + bits(dims.n_gene_ids) + bits(dims.n_umi_ids)
    return 32 + 12 + 24 * ((b + 7) // 8) + 44


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--records", type=int, default=100_000_000, help="records per rank")
    ap.add_argument("--cells", type=int, default=10_000, help="cells per rank")
    ap.add_argument("--genes", type=int, default=30_000)
    ap.add_argument("--umi-bits", type=int, default=20,
                    help="UMI ids in [0, 2^bits): 20 = 10-bp 10x v2 UMIs (default), 24 = 12-bp 10x v3")
    ap.add_argument("--float-mode", default="exact", choices=["exact", "welford"])
    ap.add_argument("--cpu-sample-s", type=float, default=15.0, help="target seconds of CPU baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="time the steps without per-kernel HIP events (no roofline / kernel table)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-check", action="store_true",
                    help="skip the record-count sanity checks (timing experimental engine builds only)")
    ap.add_argument("--config", type=int, default=None, choices=[2, 3, 4, 5],
                    help="2: cell-sorted records per rank (default at N = 1; weak scaling at N > 1); 3: ONE 100M-record "
                         "config-2 set split over the N ranks by cell ranges (default at N > 1; strong scaling); 4: the "
                         "1B-read atlas per GPU of 8 -- 125M records, 62.5k cells with lognormal(0, 2) reads; 5: globally "
                         "shuffled records, 30%% NH>1, 40%% duplicates, sorted by cell on the GPU inside every step "
                         "(SURVEY.md 8(d) configs 3, 4, 5)")
    ap.add_argument("--sort-order", default="cell_umi_gene", choices=["cell_umi_gene", "cell"],
                    help="config 5: the order sorted inside every step -- (CB, UB, GE) then query name, as "
                         "bam.sort_by_tags_and_queryname (bam.py:698-709) / TagSortBam define it (default), "
                         "or CB only (all the cell and grouped gene metrics need)")
    ap.add_argument("--traffic-json", default=None,
                    help="rocprofv3 --pmc per-kernel HBM bytes (tools/pmc_passes.sh) for roofline.traffic "
                         "(default: the committed round-5 file of this config, profiles/r05/pmc_traffic_c<N>.json)")
    a = ap.parse_args()
    if a.config is None:
        a.config = 2 if int(os.environ.get("WORLD_SIZE", "1")) == 1 else 3
    if a.traffic_json is None:  # (config 3 at N = 1 is config 2)
        a.traffic_json = os.path.join(ROOT, "profiles", "r06", "pmc_traffic_c%d.json" % (2 if a.config == 3 else a.config))
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    # rehearsal of the N-rank path on a one-GPU box (tests only, never a scaling number): every rank
    # on cuda:0, the collectives over gloo (RCCL holds one rank per device)
    share = os.environ.get("SCT_BENCH_SHARE_DEVICE") == "1"
    if share:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from sctools_amd import distributed as D
    from sctools_amd import engine as E
    from sctools_amd import synth

    eng = E.get_engine(dev)
    t0 = time.time()
    if args.config == 4:
        args.records, args.cells = 125_000_000, 62_500
    strong = args.config == 3  # one record set split over the ranks (every rank generates it, keeps its shard)
    cfg = synth.SynthConfig(n_reads=args.records, n_cells=args.cells, n_genes=args.genes,
                            sigma=2.0 if args.config == 4 else 1.0, seed=args.seed + (0 if strong else 1000 * rank),
                            umi_bits=args.umi_bits)
    if args.config == 5:  # 30 % NH > 1, 40 % duplicates, secondary alignments sharing a query name
        cfg.p_nh1, cfg.p_dup, cfg.p_secondary = 0.70, 0.40, 0.10
    data = synth.generate(cfg, device=dev, chunk=16_000_000)
    qname, n_qnames = None, 0
    n_cell_ids = data.n_cell_ids
    shard_lo, shard_hi = 0, args.records
    if strong and world > 1:  # SplitBam's cell-range shard of the one set (bam.py:361-488)
        shard_lo, shard_hi = D.shard_bounds(data.cols["cell"], world)[rank]
        data.cols = {c: t[shard_lo:shard_hi].clone() for c, t in data.cols.items()}
        torch.cuda.empty_cache()
    my_records = shard_hi - shard_lo
    if args.config == 5:  # global permutation: the step must regroup records itself
        g = torch.Generator(device=dev)
        g.manual_seed(args.seed + 1 + 1000 * rank)
        perm = torch.randperm(args.records, generator=g, device=dev)
        data.cols = {c: t[perm].contiguous() for c, t in data.cols.items()}
        qname, n_qnames = data.extra["qname"][perm].contiguous(), data.extra["n_qnames"]
        del perm
        if world > 1:
            qname, n_qnames, n_cell_ids = deal_records(data, qname, n_qnames, world, rank, dev, args.seed)
        data.extra["qname"] = qname
    torch.cuda.synchronize()
    if rank == 0:
        log("generated %d records/rank in %.1fs" % (args.records, time.time() - t0))
    dims = E.Dims(n_cell_ids, data.n_gene_ids, data.n_umi_ids)
    mito = torch.from_numpy(data.gene_is_mito).to(dev)
    multi = torch.from_numpy(data.gene_is_multi).to(dev)
    def regroup(cols):
        """config 5: TagSortBam's order on the GPU (the step's first stage); at N > 1 first the cell
        bins swapped between ranks (SplitBam's bins, bam.py:439-480): each rank then sorts its cells."""
        tie = qname
        if world > 1:
            binned, btie, counts = eng.bin_records(cols, dims, world, qname if args.sort_order != "cell" else None)
            cols, tie, _ = D.exchange_records(binned, btie, counts)
            del binned, btie
        if args.sort_order == "cell":
            return eng.tag_sort(cols, dims, "cell")
        return eng.tag_sort(cols, dims, "cell_umi_gene", tie, n_qnames)

    if args.config == 5:
        n_ent = eng.count_entities(regroup(data.cols), "cell", dims)
    else:
        n_ent = eng.count_entities(data.cols, "cell", dims)
    partials = torch.empty((data.n_gene_ids, 64), dtype=torch.int64, device=dev)
    host_cells = torch.empty((n_ent, 24), dtype=torch.int64, pin_memory=True)
    host_cellf = torch.empty((n_ent, 12), dtype=torch.float64, pin_memory=True)
    host_genei = torch.empty((data.n_gene_ids, 24), dtype=torch.int64, pin_memory=True)
    host_genef = torch.empty((data.n_gene_ids, 12), dtype=torch.float64, pin_memory=True)

    copy_stream = torch.cuda.Stream(device=dev)

    def step():
        cols = regroup(data.cols) if args.config == 5 else data.cols
        if args.float_mode == "exact":
            # one pass: cell rows + grouped gene partials share the cell-view sort
            ci, cf, _ = eng.cell_and_gene(cols, dims, mito, n_entities=n_ent, partials=partials)
        else:
            ci, cf = eng.compute(cols, "cell", dims, mito, multi, float_mode=args.float_mode, n_entities=n_ent)
            eng.gene_partials(cols, dims, out=partials)
        D.allreduce_partials(partials)  # RCCL over xGMI when N > 1; no-op at N = 1
        gi, gf = eng.finalize_partials(partials)
        # rows -> pinned host on a copy stream: this step's D2H overlaps the next step's kernels
        copy_stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(copy_stream):
            for src, dst in ((ci, host_cells[: ci.shape[0]]), (cf, host_cellf[: cf.shape[0]]), (gi, host_genei),
                             (gf, host_genef)):
                src.record_stream(copy_stream)
                dst.copy_(src, non_blocking=True)
        return ci.shape[0]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # Untimed profiling pass: HIP events around every kernel give the per-kernel table and the
    # dominant kernel.  Bracketing every launch costs ~0.3 ms per step, so the timed steps carry
    # events on the dominant kernel only (its average launch time is measured live there).
    eng.profile_only("")
    eng.profile_enable(True)
    for _ in range(PROFILE_STEPS):
        step()
    torch.cuda.synchronize()
    eng.profile_enable(False)
    table = eng.profile_read_items()
    dom_name = max(table.items(), key=lambda kv: kv[1][0])[0] if table else ""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.profile_only(dom_name)
    eng.profile_enable(not args.no_kernel_events and bool(dom_name))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rows = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    eng.profile_enable(False)
    eng.profile_only("")
    prof = eng.profile_read_items()
    elapsed = t1 - t0
    allreduce_ms = time_allreduce(partials, dev) if world > 1 else None
    step_cols = regroup(data.cols) if args.config == 5 else data.cols  # (every rank: a collective at N > 1)
    side = side_measurements(eng, data, dims, mito, multi, args, step_cols) if rank == 0 else {}
    del step_cols
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # sanity: every record accounted on both sides (config 5 at N > 1: each rank's cells after the swap)
    n_cell_reads = int(host_cells[:rows, 0].sum())
    if world > 1 and args.config == 5:
        t = torch.tensor([n_cell_reads], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        n_cell_reads = int(t.item()) // world
    if strong and world > 1:  # the shards' cell rows together cover the one set
        t = torch.tensor([n_cell_reads], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        n_cell_reads = int(t.item())
    job_records = args.records if strong else args.records * world
    if not args.no_check:
        assert n_cell_reads == (my_records if not strong else args.records), (n_cell_reads, args.records)
        assert int(host_genei[:, 0].sum()) == job_records

    total_records = job_records * args.steps
    value = total_records / elapsed
    # dominant kernel: largest total in the profiling pass; its average launch time comes from the HIP
    # events that bracketed only its launches in the timed region (on its launch stream)
    # (items: what its launches processed -- records, segment records, sort items -- as the engine
    # reports them per launch; the records of the shard where a launch does not report them)
    dom_ms, dom_launches, dom_items = prof.get(dom_name, (0.0, 1, -1))
    avg_s = dom_ms / 1e3 / max(1, dom_launches)
    items_per_launch = dom_items / max(1, dom_launches) if dom_items >= 0 else float(my_records)
    per_launch_bytes = ALG_BYTES.get(dom_name, 0) * items_per_launch
    achieved = per_launch_bytes / avg_s if avg_s > 0 else 0.0
    roofline = {
        "bound": "hbm",
        "kernel": dom_name,
        "achieved": achieved / 1e9,
        "peak": PEAK_HBM / 1e9,
        "unit": "GB/s",
        "frac": achieved / PEAK_HBM,
        "traffic": None,
        "traffic_source": None,
        "avg_launch_ms": avg_s * 1e3,
        "launches_per_step": dom_launches / args.steps,
        "alg_bytes_per_item": ALG_BYTES.get(dom_name, 0),
        "items_per_launch": items_per_launch,
        "items_source": "engine (per launch)" if dom_items >= 0 else "records of the shard",
    }
    # SURVEY.md 8(d)'s model of a sort pipeline (B_alg = 32 + 12 + 24*P + 44 bytes/record: a 7-pass LSD
    # sort that this pipeline does NOT run) -- a yardstick kept outside `roofline`, not a measured fraction
    sort_model = {"note": "SURVEY.md 8(d) 7-pass LSD sort model; not this pipeline's traffic, not measured",
                  "model_256B_alg_bytes_per_record": pipeline_bytes(args, dims),
                  "model_256B_frac": value / world * pipeline_bytes(args, dims) / PEAK_HBM}
    traffic = pmc_traffic(args, dom_name)
    if traffic is not None:
        roofline["traffic"], roofline["traffic_source"] = traffic
    # the whole step's measured HBM bytes: PMC bytes per launch x launches per step, every kernel
    step_traffic = pmc_step_traffic(args, table)
    if step_traffic is not None:
        roofline["step_traffic_bytes"] = step_traffic
        roofline["step_traffic_frac"] = step_traffic / (elapsed / args.steps) / PEAK_HBM
    kernel_ms_per_step = {k: round(v[0] / PROFILE_STEPS, 4) for k, v in sorted(table.items(), key=lambda kv: -kv[1][0])}
    kernel_items_per_step = {k: (v[2] / PROFILE_STEPS if v[2] >= 0 else None) for k, v in table.items()}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(data, args)

    if rank == 0:
        out = {
            "metric": "aligned records/sec for cell+gene metrics",
            "value": value,
            "unit": "records/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (SURVEY.md 8(d) config-%d generator, generated on GPU)" % args.config,
            "config": {
                "workload": ({2: "config2: %d cell-sorted records/rank",
                              3: "config3: ONE set of %d cell-sorted records split over the ranks by cell ranges "
                                 "balanced by records (SplitBam's invariant)",
                              4: "config4: %d cell-sorted records/rank, lognormal(0, 2) reads per cell",
                              5: "config5: %d globally shuffled records/rank (30%% NH>1, 40%% dup, secondary alignments), "
                                 + ("records of every rank's cells dealt to every rank, cell bins swapped over RCCL "
                                    "each step, then " if world > 1 else "")
                                 + "GPU sort by " + ("(CB, UB, GE, query name)" if args.sort_order != "cell" else "CB")}
                             [args.config]) % args.records + ", %d cells%s, %d genes; cell metrics + grouped gene metrics%s"
                            % (args.cells, "" if strong else "/rank", args.genes, " + RCCL all-reduce" if world > 1 else ""),
                "records_per_rank": my_records if strong else args.records,
                "records_per_job": job_records,
                "cells_per_rank": args.cells,
                "genes": args.genes,
                "float_mode": args.float_mode,
                "umi_bits": args.umi_bits,
                "parallelism": "cell-sharded x%d" % world + (" (rehearsal: ranks share cuda:0, gloo)" if share else ""),
            },
            "roofline": roofline,
            "sort_model_yardstick": sort_model,
            "kernel_ms_per_step": kernel_ms_per_step,
            "kernel_items_per_step": kernel_items_per_step,
            "kernel_table_source": "untimed profiling pass of %d steps (HIP events around every kernel)" % PROFILE_STEPS,
            "cpu_baseline": cpu,
            "speedup_vs_cpu_baseline": (value / cpu["value"]) if cpu else None,
            "reference_python": REFERENCE_PYTHON,
            "allreduce_ms": allreduce_ms,
            # the job's gene rows (all ranks' partials summed): equal for config 2 at N = 1 and config 3
            # at any N (exact-sum lanes), a check of the strong-scaling split
            "gene_rows_sha256": hashlib.sha256(host_genei.numpy().tobytes() + host_genef.numpy().tobytes()).hexdigest(),
        }
        out.update(side)
        if "h2d" in side:
            per_step_s = elapsed / args.steps + (side["h2d"]["ms"] + side["count_entities_ms"]) / 1e3
            out["records_per_s_incl_h2d_and_count"] = job_records / per_step_s
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def deal_records(data, qname, n_qnames, world, rank, dev, seed):
    """config 5 at N > 1 (setup, untimed): one globally shuffled record set over the ranks.  Each
    rank's generated cells get global ids (rank r's cells follow rank r - 1's) and its query-name
    ranks a global offset; its shuffled records are cut into `world` equal pieces and piece q goes
    to rank q (all_to_all), and every rank shuffles what it received.  So every rank holds records
    of every rank's cells in no order, and each step must swap the cell bins before it can sort.
    Returns (qname, total query names, global cell ids)."""
    from sctools_amd import distributed as D

    n = data.cols["cell"].numel()
    nq = torch.tensor([n_qnames], dtype=torch.int64, device=dev)
    all_nq = [torch.zeros_like(nq) for _ in range(world)]
    dist.all_gather(all_nq, nq)
    all_nq = [int(x.item()) for x in all_nq]
    data.cols["cell"] = data.cols["cell"] + rank * data.n_cell_ids  # (every rank: the same cell count)
    qname = qname + int(sum(all_nq[:rank]))
    piece = torch.tensor([n * (q + 1) // world - n * q // world for q in range(world)], dtype=torch.int64,
                         device=dev)
    cols, qname, _ = D.exchange_records(data.cols, qname, piece)
    g = torch.Generator(device=dev)
    g.manual_seed(seed + 7 + 1000 * rank)
    perm = torch.randperm(cols["cell"].numel(), generator=g, device=dev)
    data.cols = {c: t[perm].contiguous() for c, t in cols.items()}
    return qname[perm].contiguous(), int(sum(all_nq)), data.n_cell_ids * world


def side_measurements(eng, data, dims, mito, multi, args, cols):
    """Costs kept OUT of `value`, reported beside it:
    * the H2D copy of the 32-B SoA columns from pinned host memory (the bench generates its
      shard in HBM; a caller handing over host buffers pays this once per shard);
    * the two-phase API's sct_count_entities call (sizes the output rows; the timed steps reuse
      its answer, legitimately so for resident inputs);
    * the drop-in default: GatherCellMetrics' Welford float mode (byte-identical to the
      reference) on the same shard, cell rows only."""
    out = {}
    nbytes = sum(t.numel() * t.element_size() for t in data.cols.values())
    pinned = {c: torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for c, t in data.cols.items()}
    for c, t in data.cols.items():
        pinned[c].copy_(t)
    dst = {c: torch.empty_like(t) for c, t in data.cols.items()}
    for c in dst:  # warm
        dst[c].copy_(pinned[c], non_blocking=True)
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        for c in dst:
            dst[c].copy_(pinned[c], non_blocking=True)
    torch.cuda.synchronize()
    h2d_s = (time.perf_counter() - t0) / reps
    del dst, pinned
    out["h2d"] = {"ms": h2d_s * 1e3, "bytes": nbytes, "GB_per_s": nbytes / h2d_s / 1e9,
                  "note": "pinned host -> HBM copy of the SoA columns; excluded from value"}
    eng.count_entities(cols, "cell", dims)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        n_ent = eng.count_entities(cols, "cell", dims)
    out["count_entities_ms"] = (time.perf_counter() - t0) / reps * 1e3
    eng.compute(cols, "cell", dims, mito, multi, float_mode="welford", n_entities=n_ent)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2):
        eng.compute(cols, "cell", dims, mito, multi, float_mode="welford", n_entities=n_ent)
    torch.cuda.synchronize()
    out["dropin_cell_welford_ms"] = (time.perf_counter() - t0) / 2 * 1e3
    return out


def time_allreduce(partials, dev, reps=20):
    """The gene-partial all-reduce alone (RCCL over xGMI, [n_gene_ids, 64] int64), ms per call:
    the collective's cost beside records/s (its result is discarded: partials are re-summed)."""
    from sctools_amd import distributed as D

    buf = partials.clone()
    D.allreduce_partials(buf)
    torch.cuda.synchronize()
    dist.barrier()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        D.allreduce_partials(buf)
    b.record()
    torch.cuda.synchronize()
    t = torch.tensor([a.elapsed_time(b) / reps], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _traffic_file(args):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import source_hash

    path = args.traffic_json
    if not path or not os.path.exists(path):
        return None
    d = json.load(open(path))
    if d.get("source_sha256") != source_hash(ROOT):
        return None
    # the probe's workload must be this run's: tools/pmc_probe.py --config N at the config's sizes
    w = d.get("workload", "")
    cfg = int(w.split("--config ")[1].split()[0].rstrip(":")) if "--config " in w else 2
    sizes = {2: (100_000_000, 10_000), 4: (125_000_000, 62_500), 5: (100_000_000, 10_000)}[cfg]
    ours = 2 if args.config == 3 and int(os.environ.get("WORLD_SIZE", "1")) == 1 else args.config
    if cfg != ours or (args.records, args.cells) != sizes:
        return None
    return d


def pmc_step_traffic(args, table):
    """HBM bytes of one step: every engine kernel's PMC bytes per launch (the committed rocprofv3 --pmc
    summary of this engine source) times its launches per step (the profiling pass); None if any
    kernel of the step has no PMC figure."""
    d = _traffic_file(args)
    if d is None:
        return None
    tot = 0.0
    for k, v in table.items():
        b = pmc_bytes_per_launch(d, k)
        if b is None:
            return None
        tot += b * v[1] / PROFILE_STEPS
    return tot


def pmc_traffic(args, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary
    (tools/pmc_passes.sh -> tools/pmc_traffic.py), if it was measured on this engine source and
    this workload; else None (the roofline then reports traffic null)."""
    d = _traffic_file(args)
    b = pmc_bytes_per_launch(d, kernel) if d is not None else None
    if b is None:
        return None
    return b, os.path.relpath(args.traffic_json, ROOT)


def cpu_baseline(data, args):
    """Oracle (C restatement, OpenMP over entities) on a bounded leading sample of the shard."""
    from oracle import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    cols = data.cols
    cell = cols["cell"]

    def sample(n):
        n = min(n, cell.numel())
        if args.config == 5:  # shuffled shard: any leading slice is a fair sample (sorted inside run())
            h = {c: t[:n].cpu().numpy() for c, t in cols.items()}
            for c in ("gq_sum", "gq_len", "gq_gt30"):
                h[c] = h[c].view(np.uint16)
            h["_qname"] = data.extra["qname"][:n].cpu().numpy()
            return n, h
        # cut at a cell boundary so every cell in the sample is complete
        c_last = int(cell[n - 1].item())
        n = int(torch.searchsorted(cell, torch.tensor([c_last], dtype=cell.dtype, device=cell.device),
                                   right=False).item()) or n
        h = {c: t[:n].cpu().numpy() for c, t in cols.items()}
        for c in ("gq_sum", "gq_len", "gq_gt30"):
            h[c] = h[c].view(np.uint16)
        return n, h

    def run(h):
        t0 = time.perf_counter()
        if args.config == 5:  # the GPU step's sort first: numpy's stable lexsort, as sorted() orders
            if args.sort_order == "cell":
                order = np.argsort(h["cell"], kind="stable")
            else:
                order = np.lexsort((h["_qname"], h["gene"], h["umi"], h["cell"]))
            h = {c: a[order] for c, a in h.items() if c != "_qname"}
        O.run(h, "cell", data.gene_is_mito, data.n_gene_ids, threads=threads)
        O.run(h, "gene_grouped", data.gene_is_mito, data.n_gene_ids, threads=threads)
        return time.perf_counter() - t0

    n0, h0 = sample(2_000_000)
    t_probe = run(h0)
    rate = n0 / max(t_probe, 1e-6)
    n1, h1 = sample(int(min(cell.numel(), rate * args.cpu_sample_s)))
    t1 = run(h1)
    return {
        "value": n1 / t1,
        "unit": "records/s",
        "cores": threads,
        "kind": "port",
        "sample": ("first %d records (%d whole cells) of rank 0's shard: oracle cell metrics + grouped gene "
                   "metrics, %.1fs" % (n1, int(h1["cell"][-1]) + 1, t1)) if args.config != 5 else
                  ("first %d records of rank 0's shuffled shard: numpy stable %s + oracle cell metrics + "
                   "grouped gene metrics, %.1fs" % (n1, "sort by cell" if args.sort_order == "cell" else
                                                    "lexsort by (CB, UB, GE, query name)", t1)),
    }


if __name__ == "__main__":
    main()
