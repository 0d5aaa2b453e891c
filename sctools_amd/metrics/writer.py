"""
Metric writer -- same interface and file format as the reference's
``MetricCSVWriter`` (``/root/reference/src/sctools/metrics/writer.py:27-107``):
the stem gets ``.csv.gz`` (gzip, text mode) or ``.csv``; the header is the
mapping's public keys prefixed by an empty index column; each row is
``index,str(v)...`` with ``None`` written as ``None``.

``write_rows`` is the bulk path used by the gatherers: it writes engine
output rows without building one Python mapping per entity.
"""

import gzip
from typing import Any, Iterable, List, Mapping, Optional, TextIO


class MetricCSVWriter:
    def __init__(self, output_stem: str, compress=True):
        if compress:
            if not output_stem.endswith(".csv.gz"):
                output_stem += ".csv.gz"
        else:
            if not output_stem.endswith(".csv"):
                output_stem += ".csv"
        self._filename: str = output_stem
        if compress:
            self._open_fid: TextIO = gzip.open(self._filename, "wt")
        else:
            self._open_fid = open(self._filename, "w")
        self._header: Optional[List[str]] = None

    @property
    def filename(self) -> str:
        """filename with the suffix added"""
        return self._filename

    def write_header(self, record: Mapping[str, Any]) -> None:
        self._header = [key for key in record.keys() if not key.startswith("_")]
        self._open_fid.write("," + ",".join(self._header) + "\n")

    def write(self, index, record: Mapping[str, Any]) -> None:
        fields = [str(record[k]) for k in self._header]
        name = "None" if index is None else index
        if not isinstance(name, str):
            name = repr(name)
        self._open_fid.write(name + "," + ",".join(fields) + "\n")

    def write_rows(self, lines: Iterable[str]) -> None:
        """Write pre-formatted CSV lines (each ending in a newline)."""
        w = self._open_fid.write
        buf = []
        for line in lines:
            buf.append(line)
            if len(buf) >= 4096:
                w("".join(buf))
                buf.clear()
        if buf:
            w("".join(buf))

    def close(self) -> None:
        self._open_fid.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
