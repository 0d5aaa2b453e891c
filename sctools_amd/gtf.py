"""
GTF annotation readers (host side): mitochondrial gene ids for the cell metrics, and the
gene-name -> column map of the count matrix.

Same contract as the reference's ``sctools.gtf.get_mitochondrial_gene_names``
(``/root/reference/src/sctools/gtf.py:264-301``): every ``gene`` record whose
``gene_name`` matches ``^mt-`` (case-insensitive) contributes its ``gene_id``;
a gene record without ``gene_name`` raises ``ValueError``.  Attribute parsing
follows ``GTFRecord.__init__`` (gtf.py:84-97): field 9 split on ';', each
piece stripped and split at the first space, the value stripped of quotes.
Plain, gzip and bzip2 files are accepted (``reader.infer_open``).
"""

import bz2
import gzip
import logging
import re
import sys
from typing import Dict, Iterable, List, Set, Union

_logger = logging.getLogger(__name__)

_MT = re.compile("^mt-", re.IGNORECASE)


def _open(path: str):
    if path == "-":
        return sys.stdin
    with open(path, "rb") as f:
        magic = f.read(3)
    if magic[:2] == b"\x1f\x8b":
        return gzip.open(path, "rt")
    if magic == b"BZh":
        return bz2.open(path, "rt")
    return open(path, "r")


def _records(files: Union[str, List[str]], header_comment_char: str = "#") -> Iterable[List[str]]:
    for path in ([files] if isinstance(files, str) else list(files)):
        fh = _open(path)
        try:
            for line in fh:
                if header_comment_char and line.startswith(header_comment_char):
                    continue
                fields = line.strip(";\n").split("\t")
                if len(fields) < 9:
                    continue
                yield fields
        finally:
            if fh is not sys.stdin:
                fh.close()


def _attributes(field9: str) -> dict:
    out = {}
    for piece in field9.split(";"):
        key, _, value = piece.strip().partition(" ")
        out[key] = value.strip('"')
    return out


def get_mitochondrial_gene_names(files: Union[str, List[str]] = "-", mode: str = "r",
                                 header_comment_char: str = "#") -> Set[str]:
    """Set of gene ids of ``^mt-`` genes (the mito set passed to GatherCellMetrics)."""
    ids: Set[str] = set()
    for fields in _records(files, header_comment_char):
        if fields[2] != "gene":
            continue
        attrs = _attributes(fields[8])
        name = attrs.get("gene_name")
        if name is None:
            raise ValueError("Malformed GTF file detected. Record is of type gene but does not have a "
                             '"gene_name" field: %s' % "\t".join(fields))
        if _MT.match(name):
            ids.add(attrs.get("gene_id"))
    return ids


def _gene_records(files, header_comment_char):
    for fields in _records(files, header_comment_char):
        if fields[2] != "gene":
            continue
        attrs = _attributes(fields[8])
        name = attrs.get("gene_name")
        if name is None:
            raise ValueError("Malformed GTF file detected. Record is of type gene but does not have a "
                             '"gene_name" field: %s' % "\t".join(fields))
        yield fields, name


def _resolve_multiple_gene_names(gene_name: str) -> None:
    _logger.warning('Multiple entries encountered for "%s". Please validate the input GTF file(s). Skipping the '
                    "record for now; in the future, this will be considered as a malformed GTF file." % gene_name)


def extract_gene_names(files: Union[str, List[str]] = "-", mode: str = "r",
                       header_comment_char: str = "#") -> Dict[str, int]:
    """Gene name -> count-matrix column, in order of first occurrence among ``gene`` records; a
    repeated name is skipped with a warning (reference gtf.py:304-340)."""
    index: Dict[str, int] = {}
    for _, name in _gene_records(files, header_comment_char):
        if name in index:
            _resolve_multiple_gene_names(name)
            continue
        index[name] = len(index)
    return index


def extract_extended_gene_names(files: Union[str, List[str]] = "-", mode: str = "r",
                                header_comment_char: str = "#") -> Dict[str, List[tuple]]:
    """Chromosome -> [((start, end), gene name)] sorted by start (reference gtf.py:343-391, including
    its duplicate test against the chromosome keys).  CreateCountMatrix -n computes it; the count
    itself does not use it (count.py:240-241), here as in the reference."""
    by_chrom: Dict[str, Dict[str, tuple]] = {}
    for fields, name in _gene_records(files, header_comment_char):
        if name in by_chrom:
            _resolve_multiple_gene_names(name)
            continue
        by_chrom.setdefault(fields[0], {})[name] = (int(fields[3]), int(fields[4]))
    out: Dict[str, List[tuple]] = {}
    for chrom, genes in by_chrom.items():
        out[chrom] = sorted(((loc, name) for name, loc in genes.items()), key=lambda x: x[0])
    return out
