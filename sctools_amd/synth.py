"""
Synthetic 10x-v2-shaped columnar records (SURVEY.md §8(d), config 2 recipe).

The generator emits the 32-byte-per-record SoA layout of ``sctools_amd.columnar``
directly, so the bench never decodes a BAM.  It is written with torch tensor
ops so the same code generates small fixtures on the CPU and the 100M-record
bench workload on the GPU (torch is plumbing here; the metric kernels are the
HIP code in ``sctools_amd/csrc``).  CPU and GPU torch RNG streams differ, so a
seed names a distribution, not a bit pattern across devices; every parity
check runs the oracle on the data it actually generated.

Distributions:
* reads per cell ~ multinomial over lognormal(0, sigma) weights, cell-sorted;
* reads per molecule ~ Geometric(p=0.35); one UB (uniform 10-mer) and one GE
  per molecule; GE ~ Zipf(s=1.1) over ``n_genes``; 6 % of molecules without
  GE, 1 % with a multi-gene ``"Gx,G00000"`` value;
* ref ~ U{0..24}; pos = molecule anchor U[0, 2^27) + 50*U{0..3};
* 5 % unmapped (ref -1, no XF); mapped: 70 % reverse, 16 % duplicate,
  XF in {CODING .85, INTRONIC .05, UTR .03, INTERGENIC .07},
  NH == 1 for 90 %, 5 % spliced;
* read length 98, 13 % soft-clipped by 1-29 bases; CY 16, UY 10; binned
  Phred values with the measured per-bin weights of ``small-cell-sorted.bam``;
* CR != CB for 1 %, UR != UB for 0.2 %;
* config 5 (``p_secondary`` > 0): a record may be a secondary alignment of the record before it
  in its molecule: same query name, cell barcode and UMI, another reference, both NH > 1.
  ``extra["qname"]`` holds every record's query-name rank (names "Q%010d" of the primary's
  ordinal, so the rank is that ordinal) and ``extra["n_qnames"]`` their number.
"""

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from sctools_amd import columnar as col

PHRED_BINS = [2, 8, 12, 22, 27, 32, 37, 41]
W_GENOMIC = [3, 427, 5416, 3969, 4536, 7514, 12909, 29514]
W_CY = [1, 0, 59, 33, 102, 1578, 2253, 6470]
W_UY = [0, 0, 25, 35, 47, 105, 353, 5995]

READ_LEN, CY_LEN, UY_LEN = 98, 16, 10
N_MITO = 13


@dataclass
class SynthConfig:
    n_reads: int = 1_000_000
    n_cells: int = 100
    n_genes: int = 30_000
    sigma: float = 1.0
    seed: int = 0
    p_none_gene: float = 0.06
    p_multi_gene: float = 0.01
    p_unmapped: float = 0.05
    p_reverse: float = 0.70
    p_dup: float = 0.16
    p_nh1: float = 0.90
    p_spliced: float = 0.05
    p_softclip: float = 0.13
    p_bad_cb: float = 0.01
    p_bad_ub: float = 0.002
    p_none_cell_reads: float = 0.0  # fraction of reads emitted as a leading CB=None run
    p_secondary: float = 0.0  # records that are a secondary alignment of the previous read (config 5)
    umi_bits: int = 20  # UMI ids uniform in [0, 2^umi_bits): 20 = 10-bp 10x v2 UMIs, 24 = 12-bp 10x v3
    keep_qualities: bool = False  # keep per-base aligned qualities (fixtures only)


@dataclass
class SynthData:
    cols: Dict[str, torch.Tensor]
    n_cell_ids: int
    n_gene_ids: int
    n_umi_ids: int
    gene_names: List[Optional[str]]
    gene_is_mito: np.ndarray
    gene_is_multi: np.ndarray
    cell_has_none: bool
    quals: Optional[torch.Tensor] = None  # [n, READ_LEN] uint8 aligned qualities (padded)
    extra: dict = field(default_factory=dict)

    def cell_name(self, cid: int) -> Optional[str]:
        if self.cell_has_none:
            if cid == 0:
                return None
            cid -= 1
        return cell_barcode_string(cid)

    @staticmethod
    def umi_name(uid: int) -> str:
        return umi_string(uid)


def cell_barcode_string(i: int) -> str:
    x = (i * 0x9E3779B1 + 12345) & 0xFFFFFFFF
    s = []
    for _ in range(16):
        s.append("ACGT"[x & 3])
        x = (x >> 2) | ((x & 3) << 30)
        x = (x * 1103515245 + 12345) & 0xFFFFFFFF
    return "".join(s) + "-%d" % (i % 7)


def umi_string(u: int) -> str:
    return "".join("ACGT"[(u >> (2 * (9 - k))) & 3] for k in range(10))


def gene_dictionary(n_genes: int):
    """Sorted gene dictionary: id 0 is None, then names in string order.

    Returns (names, rank_to_id, multi_rank_to_id, mito_flags, multi_flags):
    Zipf rank r (0-based) maps to gene ``G%05d % r``; its multi-gene variant
    ``G%05d,G00000`` is a distinct dictionary entry.
    """
    singles = ["G%05d" % r for r in range(n_genes)]
    multis = ["G%05d,G00000" % r for r in range(n_genes)]
    names_sorted = sorted(singles + multis)
    index = {n: i + 1 for i, n in enumerate(names_sorted)}
    names: List[Optional[str]] = [None] + names_sorted
    rank_to_id = np.array([index[s] for s in singles], dtype=np.int64)
    multi_rank_to_id = np.array([index[m] for m in multis], dtype=np.int64)
    mito = np.zeros(len(names), dtype=np.uint8)
    for r in mito_ranks(n_genes):
        mito[rank_to_id[r]] = 1
    multi = np.array([1 if (n is not None and "," in n) else 0 for n in names], dtype=np.uint8)
    return names, rank_to_id, multi_rank_to_id, mito, multi


def mito_ranks(n_genes: int) -> List[int]:
    cand = [3, 9, 17, 28, 44, 71, 112, 180, 290, 470, 760, 1230, 1990]
    return [c for c in cand if c < n_genes][:N_MITO]


def _bin_sampler(weights, device):
    w = torch.tensor(weights, dtype=torch.float64)
    cdf = torch.cumsum(w / w.sum(), 0)
    cdf[-1] = 1.0
    return cdf.to(device=device, dtype=torch.float32), torch.tensor(
        PHRED_BINS, dtype=torch.int32, device=device
    )


def _sample_quals(gen, n, length, weights, device):
    cdf, vals = _bin_sampler(weights, device)
    u = torch.rand((n, length), generator=gen, device=device, dtype=torch.float32)
    idx = torch.bucketize(u, cdf, right=True).clamp_(max=len(PHRED_BINS) - 1)
    return vals[idx]


def generate(cfg: SynthConfig, device="cpu", chunk: int = 8_000_000) -> SynthData:
    """Generate ``cfg.n_reads`` cell-sorted records as columnar tensors on ``device``."""
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(cfg.seed)
    n = int(cfg.n_reads)

    names, rank_to_id, multi_rank_to_id, gene_is_mito, gene_is_multi = gene_dictionary(cfg.n_genes)
    # --- reads per cell: multinomial over lognormal weights ---
    cgen = torch.Generator()
    cgen.manual_seed(cfg.seed + 1)
    w = torch.exp(torch.randn(cfg.n_cells, generator=cgen, dtype=torch.float64) * cfg.sigma)
    n_none = int(round(n * cfg.p_none_cell_reads))
    n_cellreads = n - n_none
    counts = torch.multinomial(w / w.sum(), n_cellreads, replacement=True, generator=cgen)
    per_cell = torch.bincount(counts, minlength=cfg.n_cells)
    has_none = n_none > 0
    # cell id per read (cell-sorted; optional leading None run gets id 0)
    cell_ids = torch.arange(cfg.n_cells, dtype=torch.int32) + (1 if has_none else 0)
    cell = torch.repeat_interleave(cell_ids, per_cell)
    if has_none:
        cell = torch.cat([torch.zeros(n_none, dtype=torch.int32), cell])
    cell = cell.to(dev)

    # --- molecules: geometric(0.35) reads per molecule, packed inside each cell ---
    # Draw molecule lengths as a stream and cut them at cell boundaries.
    seg_sizes = torch.cat([torch.tensor([n_none], dtype=torch.int64), per_cell.to(torch.int64)])
    seg_sizes = seg_sizes[seg_sizes > 0]
    seg_start = torch.cumsum(seg_sizes, 0) - seg_sizes
    # molecule id per read: a new molecule starts at each cell start or when the geometric run ends
    p = 0.35
    u = torch.rand(n, generator=gen, device=dev, dtype=torch.float32)
    mol_head = u < p
    head_idx = seg_start.to(dev)
    mol_head[head_idx] = True
    mol_head[0] = True
    mol_id = torch.cumsum(mol_head.to(torch.int64), 0) - 1
    n_mol = int(mol_id[-1].item()) + 1

    # per-molecule attributes
    zipf_s = 1.1
    ranks = torch.arange(1, cfg.n_genes + 1, dtype=torch.float64)
    zcdf = torch.cumsum(ranks.pow(-zipf_s), 0)
    zcdf = (zcdf / zcdf[-1]).to(dev)
    mu = torch.rand(n_mol, generator=gen, device=dev, dtype=torch.float64)
    grank = torch.bucketize(mu, zcdf, right=True).clamp_(max=cfg.n_genes - 1)
    r2i = torch.from_numpy(rank_to_id).to(dev)
    mr2i = torch.from_numpy(multi_rank_to_id).to(dev)
    gsel = torch.rand(n_mol, generator=gen, device=dev, dtype=torch.float64)
    mol_gene = torch.where(gsel < cfg.p_none_gene, torch.zeros_like(grank),
                           torch.where(gsel < cfg.p_none_gene + cfg.p_multi_gene, mr2i[grank], r2i[grank]))
    mol_umi = torch.randint(0, 1 << cfg.umi_bits, (n_mol,), generator=gen, device=dev, dtype=torch.int64)
    mol_ref = torch.randint(0, 25, (n_mol,), generator=gen, device=dev, dtype=torch.int64)
    mol_anchor = torch.randint(0, 1 << 27, (n_mol,), generator=gen, device=dev, dtype=torch.int64)

    gene = mol_gene[mol_id].to(torch.int32)
    umi = mol_umi[mol_id].to(torch.int32)
    ref = mol_ref[mol_id].to(torch.int32)
    pos = (mol_anchor[mol_id] + 50 * torch.randint(0, 4, (n,), generator=gen, device=dev)).to(torch.int32)
    # secondary alignments: a non-head record of a molecule may repeat the previous record's read
    # (same query name, CB, UB) at another locus; both then have NH > 1
    qname = None
    secondary = None
    if cfg.p_secondary > 0:
        secondary = (torch.rand(n, generator=gen, device=dev) < cfg.p_secondary) & ~mol_head
        qname = (torch.cumsum((~secondary).to(torch.int64), 0) - 1).to(torch.int32)
        shift = torch.randint(1, 25, (n,), generator=gen, device=dev, dtype=torch.int64)
        ref = torch.where(secondary, ((ref.to(torch.int64) + shift) % 25).to(torch.int32), ref)
        del shift
    del mol_id, mol_head, mu, grank, gsel

    def bern(prob):
        return torch.rand(n, generator=gen, device=dev) < prob

    unmapped = bern(cfg.p_unmapped)
    reverse = bern(cfg.p_reverse) & ~unmapped
    dup = bern(cfg.p_dup) & ~unmapped
    spliced = bern(cfg.p_spliced) & ~unmapped
    nh1 = bern(cfg.p_nh1)
    if secondary is not None:  # a multi-mapped read: the primary and its secondaries have NH > 1
        multi = secondary.clone()
        multi[:-1] |= secondary[1:]
        nh1 &= ~multi
        del multi
    perfect_umi = ~bern(cfg.p_bad_ub)
    has_cb = (cell != 0) if has_none else torch.ones(n, dtype=torch.bool, device=dev)
    perfect_cb = has_cb & ~bern(cfg.p_bad_cb)
    ref = torch.where(unmapped, torch.full_like(ref, -1), ref)
    pos = torch.where(unmapped, torch.full_like(pos, -1), pos)
    xr = torch.rand(n, generator=gen, device=dev)
    xf = torch.full((n,), col.XF_CODING, dtype=torch.uint8, device=dev)
    xf = torch.where(xr >= 0.85, torch.full_like(xf, col.XF_INTRONIC), xf)
    xf = torch.where(xr >= 0.90, torch.full_like(xf, col.XF_UTR), xf)
    xf = torch.where(xr >= 0.93, torch.full_like(xf, col.XF_INTERGENIC), xf)
    xf = torch.where(unmapped, torch.full_like(xf, col.XF_ABSENT), xf)
    bits = (
        unmapped.to(torch.uint8) * col.B_UNMAPPED
        | reverse.to(torch.uint8) * col.B_REVERSE
        | dup.to(torch.uint8) * col.B_DUPLICATE
        | spliced.to(torch.uint8) * col.B_SPLICED
        | nh1.to(torch.uint8) * col.B_NH1
        | perfect_umi.to(torch.uint8) * col.B_PERFECT_UMI
        | has_cb.to(torch.uint8) * col.B_HAS_CB
        | perfect_cb.to(torch.uint8) * col.B_PERFECT_CB
    ).to(torch.uint8)
    del unmapped, reverse, dup, spliced, nh1, perfect_umi, has_cb, perfect_cb, xr

    # --- qualities: per-base binned Phred, reduced to (sum, len, >30) in chunks ---
    clip = torch.where(bern(cfg.p_softclip),
                       torch.randint(1, 30, (n,), generator=gen, device=dev),
                       torch.zeros(n, dtype=torch.int64, device=dev))
    gq_len = (READ_LEN - clip).to(torch.int32)
    gq_sum = torch.empty(n, dtype=torch.int32, device=dev)
    gq_gt30 = torch.empty(n, dtype=torch.int32, device=dev)
    cy_gt30 = torch.empty(n, dtype=torch.int32, device=dev)
    uy_gt30 = torch.empty(n, dtype=torch.int32, device=dev)
    quals = torch.empty((n, READ_LEN), dtype=torch.uint8) if cfg.keep_qualities else None
    lane = torch.arange(READ_LEN, device=dev, dtype=torch.int32)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        q = _sample_quals(gen, e - s, READ_LEN, W_GENOMIC, dev)
        q = torch.where(lane[None, :] < gq_len[s:e, None], q, torch.zeros_like(q))
        gq_sum[s:e] = q.sum(1, dtype=torch.int32)
        gq_gt30[s:e] = (q > 30).sum(1, dtype=torch.int32)
        if quals is not None:
            quals[s:e] = q.to(torch.uint8).cpu()
        del q
        cq = _sample_quals(gen, e - s, CY_LEN, W_CY, dev)
        cy_gt30[s:e] = (cq > 30).sum(1, dtype=torch.int32)
        uq = _sample_quals(gen, e - s, UY_LEN, W_UY, dev)
        uy_gt30[s:e] = (uq > 30).sum(1, dtype=torch.int32)
        del cq, uq

    cols = {
        "cell": cell.contiguous(),
        "umi": umi.contiguous(),
        "gene": gene.contiguous(),
        "ref": ref.contiguous(),
        "pos": pos.contiguous(),
        "gq_sum": gq_sum.to(torch.int16).contiguous(),  # reinterpreted as uint16 (sum <= 98*41)
        "gq_len": gq_len.to(torch.int16).contiguous(),
        "gq_gt30": gq_gt30.to(torch.int16).contiguous(),
        "bits": bits.contiguous(),
        "xf": xf.contiguous(),
        "cy_gt30": cy_gt30.to(torch.uint8).contiguous(),
        "cy_len": torch.full((n,), CY_LEN, dtype=torch.uint8, device=dev),
        "uy_gt30": uy_gt30.to(torch.uint8).contiguous(),
        "uy_len": torch.full((n,), UY_LEN, dtype=torch.uint8, device=dev),
    }
    return SynthData(
        cols=cols,
        n_cell_ids=cfg.n_cells + (1 if has_none else 0),
        n_gene_ids=len(names),
        n_umi_ids=1 << cfg.umi_bits,
        gene_names=names,
        gene_is_mito=gene_is_mito,
        gene_is_multi=gene_is_multi,
        cell_has_none=has_none,
        quals=quals,
        extra={"per_cell": per_cell.numpy(), "n_none": n_none, "qname": qname,
               "n_qnames": int(qname[-1].item()) + 1 if qname is not None else 0},
    )


def shuffle_within_entities(cols: Dict[str, torch.Tensor], key: str, seed: int) -> Dict[str, torch.Tensor]:
    """Permute records inside each run of ``cols[key]`` (keeps run membership)."""
    k = cols[key]
    n = k.numel()
    g = torch.Generator(device=k.device)
    g.manual_seed(seed)
    run = torch.cumsum(torch.cat([torch.ones(1, dtype=torch.int64, device=k.device),
                                  (k[1:] != k[:-1]).to(torch.int64)]), 0)
    r = torch.rand(n, generator=g, device=k.device, dtype=torch.float64)
    order = torch.argsort(run.to(torch.float64) * 2.0 + r)
    return {c: v[order].contiguous() for c, v in cols.items()}
