"""
Columnar record layout and the BAM -> columns host path.

Each alignment becomes 32 bytes spread over SoA columns:

=========  ======  =====================================================
column     dtype   meaning
=========  ======  =====================================================
cell       int32   dictionary id of the CB tag (missing CB is an id too)
umi        int32   dictionary id of the UB tag (missing UB is an id too)
gene       int32   dictionary id of the GE tag (missing GE is an id too)
ref        int32   ``reference_id``
pos        int32   ``pos`` (0-based leftmost)
gq_sum     uint16  sum of ``query_alignment_qualities``
gq_len     uint16  len(``query_alignment_qualities``)
gq_gt30    uint16  #bases of ``query_alignment_qualities`` with Q > 30
bits       uint8   B_* flags below
xf         uint8   XF_* enum below
cy_gt30    uint8   #CY bases with Q > 30
cy_len     uint8   len(CY)
uy_gt30    uint8   #UY bases with Q > 30
uy_len     uint8   len(UY)
=========  ======  =====================================================

The reference reads every one of these per record inside
``MetricAggregator.parse_molecule`` (``aggregator.py:251-334``) and
``CellMetrics.parse_extra_fields`` (``aggregator.py:507-530``).  The
conversion below raises the same exception types the reference raises while
it aggregates (SURVEY.md §8(b) "Errors"), in the same record order, before
anything is handed to the device.
"""

from typing import Dict, List, Optional

import numpy as np

from sctools_amd import consts
from sctools_amd.bam import open_alignments

# bits column
B_UNMAPPED = 1 << 0  # flag & 0x4
B_REVERSE = 1 << 1  # flag & 0x10
B_DUPLICATE = 1 << 2  # flag & 0x400
B_SPLICED = 1 << 3  # CIGAR N length > 0
B_NH1 = 1 << 4  # NH == 1
B_PERFECT_UMI = 1 << 5  # UR and UB present and equal
B_HAS_CB = 1 << 6  # CB present
B_PERFECT_CB = 1 << 7  # CB present and CR == CB

# xf column
XF_ABSENT, XF_CODING, XF_INTRONIC, XF_UTR, XF_INTERGENIC, XF_OTHER = range(6)
_XF_CODE = {
    consts.CODING_ALIGNMENT_LOCATION_TAG_VALUE: XF_CODING,
    consts.INTRONIC_ALIGNMENT_LOCATION_TAG_VALUE: XF_INTRONIC,
    consts.UTR_ALIGNMENT_LOCATION_TAG_VALUE: XF_UTR,
    consts.INTERGENIC_ALIGNMENT_LOCATION_TAG_VALUE: XF_INTERGENIC,
}

COLUMNS = [
    ("cell", np.int32), ("umi", np.int32), ("gene", np.int32), ("ref", np.int32),
    ("pos", np.int32), ("gq_sum", np.uint16), ("gq_len", np.uint16), ("gq_gt30", np.uint16),
    ("bits", np.uint8), ("xf", np.uint8), ("cy_gt30", np.uint8), ("cy_len", np.uint8),
    ("uy_gt30", np.uint8), ("uy_len", np.uint8),
]
COLUMN_NAMES = [c for c, _ in COLUMNS]
BYTES_PER_RECORD = sum(np.dtype(t).itemsize for _, t in COLUMNS)  # 32

MODE_CELL = "cell"
MODE_GENE = "gene"


def _sort_key(v):
    # None first, then values in Python order (strings lexicographic)
    return (0, "") if v is None else (1, str(v))


class Dictionary:
    """Tag value <-> dense id.  ``None`` (missing tag) is an ordinary entry."""

    def __init__(self, values: List, presorted: bool = False):
        self.names: List = list(values) if presorted else sorted(set(values), key=_sort_key)
        self.index: Dict = {v: i for i, v in enumerate(self.names)}

    def __len__(self):
        return len(self.names)

    def encode(self, values: List) -> np.ndarray:
        idx = self.index
        return np.fromiter((idx[v] for v in values), dtype=np.int32, count=len(values))


class PackedDictionary:
    """A ranked dictionary as the decoders hand it over: the names' bytes back to back in id
    order, their offsets, and whether id 0 is the missing tag.  Names are decoded to ``str`` only
    when asked for (a UMI dictionary of millions of entries is needed only for its length)."""

    def __init__(self, raw: bytes, offsets: np.ndarray, has_none: bool):
        self._raw, self._off, self._has_none = raw, offsets, bool(has_none)
        self._names: Optional[List] = None
        self._index: Optional[Dict] = None

    def __len__(self):
        return len(self._off) - 1

    @property
    def names(self) -> List:
        if self._names is None:
            raw, off = self._raw, self._off.tolist()
            lst = [raw[off[i]:off[i + 1]].decode("utf-8") for i in range(len(off) - 1)]
            if self._has_none:
                lst[0] = None
            self._names = lst
        return self._names

    @property
    def index(self) -> Dict:
        if self._index is None:
            self._index = {v: i for i, v in enumerate(self.names)}
        return self._index


class Columns:
    """Columnar records plus the dictionaries needed to print entity names.  ``arrays`` holds
    numpy columns (host decode) or device tensors (``gbam``, decoded on the GPU)."""

    def __init__(self, arrays: Dict[str, np.ndarray], cells: Dictionary, umis: Dictionary,
                 genes: Dictionary):
        self.arrays = arrays
        self.cells = cells
        self.umis = umis
        self.genes = genes

    @property
    def n(self) -> int:
        return int(self.arrays["cell"].shape[0])

    @property
    def on_device(self) -> bool:
        return not isinstance(self.arrays["cell"], np.ndarray)

    def host(self) -> "Columns":
        """These columns with numpy arrays (copied from the device when they live there)."""
        if not self.on_device:
            return self
        arrays = {}
        for c, t in self.arrays.items():
            a = t.cpu().numpy()
            arrays[c] = a.view(np.uint16) if a.dtype == np.int16 else a
        return Columns(arrays, self.cells, self.umis, self.genes)

    def column_at(self, name: str, index: np.ndarray) -> np.ndarray:
        """``arrays[name][index]`` as numpy, gathered on the device for device columns."""
        a = self.arrays[name]
        if isinstance(a, np.ndarray):
            return a[index]
        import torch

        idx = torch.from_numpy(np.ascontiguousarray(index, dtype=np.int64)).to(a.device)
        return a[idx].cpu().numpy()

    def gene_flags(self, mitochondrial_gene_ids=frozenset()):
        """(is_mito, is_multi) uint8 per gene id.

        Mito membership tests the GE *string* against the GTF gene ids, as
        ``CellMetrics.finalize`` does (``aggregator.py:476-482``); multi-gene
        is a non-None GE containing ',' (``gatherer.py:210-212``).
        """
        names = self.genes.names
        mito = np.fromiter((1 if g in mitochondrial_gene_ids else 0 for g in names),
                           dtype=np.uint8, count=len(names))
        multi = np.fromiter((1 if (g and len(str(g).split(",")) > 1) else 0 for g in names),
                            dtype=np.uint8, count=len(names))
        return mito, multi


class ShardedColumns:
    """Device columns of one file held as contiguous record ranges on several devices (``gbam``'s
    per-device decode, ``GatherCellMetrics(devices=N)``): shard r holds records
    ``offsets[r] .. offsets[r + 1]`` of the file, in file order, on its device; the dictionaries
    are global.  Shards are cut at runs of ``key`` (cut_runs), so an entity never spans two."""

    on_device = True

    def __init__(self, shards: List[Dict], cells, umis, genes):
        self.shards = shards
        self.cells = cells
        self.umis = umis
        self.genes = genes

    @property
    def offsets(self) -> List[int]:
        out = [0]
        for sh in self.shards:
            out.append(out[-1] + int(sh["cell"].shape[0]))
        return out

    @property
    def n(self) -> int:
        return self.offsets[-1]

    def host(self) -> "Columns":
        """One host Columns of every shard's records, in order (tests)."""
        arrays = {}
        for c in self.shards[0]:
            parts = [sh[c].cpu().numpy() for sh in self.shards]
            a = np.concatenate(parts)
            arrays[c] = a.view(np.uint16) if a.dtype == np.int16 else a
        return Columns(arrays, self.cells, self.umis, self.genes)

    def column_at(self, name: str, index: np.ndarray) -> np.ndarray:
        """Column ``name`` at file-wide record indices, gathered on the shards' devices."""
        import torch

        index = np.asarray(index, dtype=np.int64)
        off = np.asarray(self.offsets, dtype=np.int64)
        which = np.searchsorted(off, index, side="right") - 1
        out = None
        for r, sh in enumerate(self.shards):
            sel = np.flatnonzero(which == r)
            if not sel.size:
                continue
            t = sh[name]
            idx = torch.from_numpy(index[sel] - off[r]).to(t.device)
            v = t[idx].cpu().numpy()
            if out is None:
                out = np.empty(index.shape[0], dtype=v.dtype)
            out[sel] = v
        if out is None:
            out = np.empty(0, dtype=np.int32)
        return out

    gene_flags = Columns.gene_flags


def cut_runs(shards: List[Dict], key: str) -> List[Dict]:
    """Shards re-cut so that no run of equal ``key`` values spans two: the records at the head of a
    shard continuing the previous (non-empty) shard's last run move to the end of that shard --
    SplitBam's invariant (bam.py:439-448), an entity's records on one device.  Columns moved or
    left behind are fresh 16-byte-aligned buffers (the kernels' vector loads need them)."""
    import torch

    shards = [dict(sh) for sh in shards]
    prev = None
    for r in range(len(shards)):
        sh = shards[r]
        n = int(sh[key].shape[0])
        if n == 0:
            continue
        if prev is not None:
            # host values: the two shards may live on different devices
            last = int(shards[prev][key][-1].item())
            col = sh[key]
            if int(col[0].item()) == last:
                diff = torch.nonzero(col != col[0])
                k = int(diff[0, 0].item()) if diff.numel() else n
                dst = shards[prev][key].device
                for c in list(sh.keys()):
                    moved = sh[c][:k].to(dst)
                    shards[prev][c] = torch.cat((shards[prev][c], moved))
                    sh[c] = sh[c][k:].clone()
                if k == n:
                    continue  # the whole shard continued the run: the next one compares with prev
        prev = r
    return shards


def columnarize_parts(path: str, metric_mode: str, devices, key: str) -> Optional[ShardedColumns]:
    """A BAM decoded by ``devices`` together (``gbam.decode_parts``: part r on devices[r]), shards
    cut at runs of ``key``; None when the file needs the host decoder."""
    from sctools_amd import gbam

    got = gbam.decode_parts(path, metric_mode, devices)
    if got is None:
        return None
    shards, (cn, un, gn) = got
    return ShardedColumns(cut_runs(shards, key), cn, un, gn)


def _frac_counts(quality_string: str):
    # _quality_string_to_numeric + _quality_above_threshold (aggregator.py:191-231)
    n = len(quality_string)
    if n == 0:
        raise ZeroDivisionError("division by zero")
    gt = 0
    for c in quality_string:
        if ord(c) - 33 > 30:
            gt += 1
    return gt, n


def record_fields(rec, cb, is_cell: bool, validate: bool):
    """Numeric columns of one record, raising like the reference would.

    Follows the per-record reads of ``CellMetrics.parse_extra_fields``
    (aggregator.py:507-527, cell mode only) and ``parse_molecule``
    (aggregator.py:266-331).  ``cb`` is the record's CB value (or None).
    Returns (ref, pos, gq_sum, gq_len, gq_gt30, bits, xf, cy_gt30, cy_len,
    uy_gt30, uy_len).
    """
    tags = rec._tags if hasattr(rec, "_tags") else None
    get = (lambda k, d=None: tags.get(k, d)) if tags is not None else (
        lambda k, d=None: rec.get_tag(k) if rec.has_tag(k) else d)
    b = 0
    cg = cl = 0
    if is_cell:
        cg, cl = _frac_counts(rec.get_tag(consts.QUALITY_CELL_BARCODE_TAG_KEY))
        if cb is not None:
            b |= B_HAS_CB
            if rec.get_tag(consts.RAW_CELL_BARCODE_TAG_KEY) == cb:
                b |= B_PERFECT_CB
    elif cb is not None:
        b |= B_HAS_CB
    if validate:
        ug, ul = _frac_counts(rec.get_tag(consts.QUALITY_MOLECULE_BARCODE_TAG_KEY))
    else:
        uyq = get(consts.QUALITY_MOLECULE_BARCODE_TAG_KEY, "")
        ug, ul = (_frac_counts(uyq) if uyq else (0, 0))
    ur = get(consts.RAW_MOLECULE_BARCODE_TAG_KEY)
    ub = get(consts.MOLECULE_BARCODE_TAG_KEY)
    if ur is not None and ub is not None and ur == ub:
        b |= B_PERFECT_UMI
    aq = rec.query_alignment_qualities
    if aq is None:
        if validate:
            raise TypeError("'NoneType' object is not iterable")
        aq = b""
    if len(aq) == 0 and validate:
        raise ZeroDivisionError("division by zero")
    x = XF_ABSENT
    xfv = get(consts.ALIGNMENT_LOCATION_TAG_KEY)
    if xfv is not None:
        x = _XF_CODE.get(xfv, XF_OTHER)
    flag = rec.flag
    if flag & 0x4:
        b |= B_UNMAPPED
    else:
        if validate:
            rec.get_tag(consts.ALIGNMENT_LOCATION_TAG_KEY)  # KeyError like aggregator.py:305
            nh = rec.get_tag(consts.NUMBER_OF_HITS_TAG_KEY)  # KeyError like aggregator.py:317
        else:
            nh = get(consts.NUMBER_OF_HITS_TAG_KEY, 0)
        if nh == 1:
            b |= B_NH1
        n_len = rec.n_skip_length() if hasattr(rec, "n_skip_length") else rec.get_cigar_stats()[0][3]
        if n_len:
            b |= B_SPLICED
    if flag & 0x10:
        b |= B_REVERSE
    if flag & 0x400:
        b |= B_DUPLICATE
    s = sum(aq)
    g = sum(1 for q in aq if q > 30)
    if len(aq) > 0xFFFF or s > 0xFFFF or cl > 0xFF or ul > 0xFF:
        raise ValueError("record %s exceeds the 32-byte columnar limits" % getattr(rec, "query_name", "?"))
    return (rec.reference_id, rec.pos, s, len(aq), g, b, x, cg, cl, ug, ul)


_NUMERIC = ("ref", "pos", "gq_sum", "gq_len", "gq_gt30", "bits", "xf", "cy_gt30", "cy_len", "uy_gt30",
            "uy_len")


def build_columns(cell_v: List, umi_v: List, gene_v: List, numeric: List[tuple]) -> Columns:
    """Dictionary-encode the tag values and pack the numeric tuples into columns."""
    cells, umis, genes = Dictionary(cell_v), Dictionary(umi_v), Dictionary(gene_v)
    arrays = {"cell": cells.encode(cell_v), "umi": umis.encode(umi_v), "gene": genes.encode(gene_v)}
    dtypes = dict(COLUMNS)
    if numeric:
        cols = list(zip(*numeric))
    else:
        cols = [[] for _ in _NUMERIC]
    for name, values in zip(_NUMERIC, cols):
        arrays[name] = np.asarray(values, dtype=dtypes[name])
    return Columns(arrays, cells, umis, genes)


def columnarize(path: str, mode: str = "rb", metric_mode: str = MODE_CELL, native: Optional[bool] = None,
                device=None) -> Columns:
    """Decode ``path`` into :class:`Columns`, validating like the reference.

    ``metric_mode`` selects which tags are required: ``cell`` also needs
    CY (and CR for reads that carry CB), as ``CellMetrics.parse_extra_fields``
    does; ``gene`` does not, and records of multi-gene GE runs are never
    validated because ``GatherGeneMetrics`` skips them (``gatherer.py:210-212``).

    With ``device`` (a torch device) a BAM is decoded on that GPU (``gbam``: inflate, record
    starts, parse and interning in HBM) and the columns stay there.  A file the device path
    declines (a record the reference rejects, typed dictionary tags) and every other case go
    through the native host decoder (``libsct_bam.so``, all cores) unless ``native=False``;
    SAM text, and BAM with ``native=False``, through the Python reader.
    """
    from sctools_amd import bamnative

    if device is not None and mode == "rb" and native is not False:
        from sctools_amd import gbam

        got = gbam.decode(path, metric_mode, device, lazy=True)
        if got is not None:
            arrays, (cn, un, gn) = got
            return Columns(arrays, cn, un, gn)
    if native is None:
        native = mode == "rb" and bamnative.available()
    if native:
        if mode != "rb":
            raise ValueError("the native decoder reads BAM (mode 'rb')")
        try:
            arrays, (cn, un, gn) = bamnative.decode(path, metric_mode)
            return Columns(arrays, Dictionary(cn, True), Dictionary(un, True), Dictionary(gn, True))
        except bamnative.TypedTagValue:  # float / array CB, UB or GE values: the Python reader keys them
            pass
    cell_v, umi_v, gene_v, numeric = [], [], [], []
    is_cell = metric_mode == MODE_CELL
    prev_gene = object()
    skip_run = False
    for rec in open_alignments(path, mode):
        tags = rec._tags
        cb = tags.get(consts.CELL_BARCODE_TAG_KEY)
        ge = tags.get(consts.GENE_NAME_TAG_KEY)
        if not is_cell and ge != prev_gene:
            prev_gene = ge
            skip_run = bool(ge) and len(str(ge).split(",")) > 1
        numeric.append(record_fields(rec, cb, is_cell, is_cell or not skip_run))
        cell_v.append(cb)
        umi_v.append(tags.get(consts.MOLECULE_BARCODE_TAG_KEY))
        gene_v.append(ge)
    if not cell_v:
        # iter_tag_groups: next() on an empty iterator inside a generator (bam.py:517)
        raise RuntimeError("generator raised StopIteration")
    return build_columns(cell_v, umi_v, gene_v, numeric)


def bit_count(n: int) -> int:
    """Bits needed to hold ids 0..n-1 (at least 1)."""
    return max(1, int(n - 1).bit_length())
