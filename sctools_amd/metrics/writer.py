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
from typing import Any, Iterable, List, Mapping, Optional


class MetricCSVWriter:
    """With ``compress`` and the native library built, the text is kept in memory and gzipped at
    ``close()`` in parallel members (level 9, as the reference's ``gzip.open``); the file
    decompresses to the same text.  Otherwise it streams through ``gzip.open`` / ``open``."""

    def __init__(self, output_stem: str, compress=True):
        from sctools_amd import csvnative

        if compress:
            if not output_stem.endswith(".csv.gz"):
                output_stem += ".csv.gz"
        else:
            if not output_stem.endswith(".csv"):
                output_stem += ".csv"
        self._filename: str = output_stem
        self._parts: Optional[List[bytes]] = None
        if compress and csvnative.available():
            self._parts = []
            self._open_fid = open(self._filename, "wb")
        elif compress:
            self._open_fid = gzip.open(self._filename, "wt")
        else:
            self._open_fid = open(self._filename, "w")
        self._header: Optional[List[str]] = None

    @property
    def filename(self) -> str:
        """filename with the suffix added"""
        return self._filename

    def _emit(self, text: str) -> None:
        if self._parts is not None:
            self._parts.append(text.encode("utf-8"))
        else:
            self._open_fid.write(text)

    def write_header(self, record: Mapping[str, Any]) -> None:
        self._header = [key for key in record.keys() if not key.startswith("_")]
        self._emit("," + ",".join(self._header) + "\n")

    def write(self, index, record: Mapping[str, Any]) -> None:
        fields = [str(record[k]) for k in self._header]
        name = "None" if index is None else index
        if not isinstance(name, str):
            name = repr(name)
        self._emit(name + "," + ",".join(fields) + "\n")

    def write_rows(self, lines: Iterable[str]) -> None:
        """Write pre-formatted CSV lines (each ending in a newline)."""
        buf = []
        for line in lines:
            buf.append(line)
            if len(buf) >= 4096:
                self._emit("".join(buf))
                buf.clear()
        if buf:
            self._emit("".join(buf))

    def write_bytes(self, data: bytes) -> None:
        """Write pre-formatted UTF-8 CSV text (metrics.rows.format_rows_bytes)."""
        if self._parts is not None:
            self._parts.append(data)
        elif isinstance(self._open_fid, gzip.GzipFile) or "b" not in getattr(self._open_fid, "mode", "w"):
            self._open_fid.write(data.decode("utf-8"))
        else:
            self._open_fid.write(data)

    def close(self) -> None:
        if self._parts is not None:
            from sctools_amd import csvnative

            self._open_fid.write(csvnative.gzip(b"".join(self._parts), level=9))
            self._parts = None
        self._open_fid.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
