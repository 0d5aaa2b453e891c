"""
Stand-in ``pysam`` used ONLY by ``tests/golden/make_golden.py`` to run the
unmodified reference gatherer in the build container (pysam is not installed
and there is no network; SURVEY.md §8(c) "Verified recipe").

It exposes the surface the metric path touches: ``AlignmentFile`` (context
manager and iterator) and ``AlignedSegment`` with ``get_tag``, ``has_tag``,
``is_unmapped``, ``is_reverse``, ``is_duplicate``, ``pos``, ``reference_id``,
``get_cigar_stats`` and ``query_alignment_qualities`` (pysam 0.16
semantics, implemented in ``sctools_amd.bam``).  Synthetic fixtures build
``AlignedSegment`` objects directly from generator columns.
"""

from array import array

from sctools_amd.bam import BamRecord, open_alignments


class AlignedSegment:
    __slots__ = ("_tags", "flag", "reference_id", "pos", "query_name", "_n_len", "_aq")

    def __init__(self, tags, flag, reference_id, pos, n_len, aligned_qualities, query_name="r"):
        self._tags = tags
        self.flag = flag
        self.reference_id = reference_id
        self.pos = pos
        self.query_name = query_name
        self._n_len = n_len
        self._aq = aligned_qualities

    @classmethod
    def from_bam(cls, rec: BamRecord) -> "AlignedSegment":
        aq = rec.query_alignment_qualities
        return cls(rec._tags, rec.flag, rec.reference_id, rec.pos, rec.n_skip_length(),
                   None if aq is None else array("B", aq), rec.query_name)

    def get_tag(self, tag):
        return self._tags[tag]

    def has_tag(self, tag):
        return tag in self._tags

    @property
    def is_unmapped(self):
        return bool(self.flag & 0x4)

    @property
    def is_reverse(self):
        return bool(self.flag & 0x10)

    @property
    def is_duplicate(self):
        return bool(self.flag & 0x400)

    @property
    def query_alignment_qualities(self):
        return self._aq

    def get_cigar_stats(self):
        stats = [0] * 11
        stats[3] = self._n_len
        return stats, [0] * 11


class AlignmentFile:
    def __init__(self, path, mode="rb", **kwargs):
        if isinstance(path, list):  # pre-built segments (synthetic fixtures)
            self._it = iter(path)
        else:
            self._it = (AlignedSegment.from_bam(r) for r in open_alignments(path, mode))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def __iter__(self):
        return self

    def __next__(self):
        return next(self._it)

    def close(self):
        pass


def merge(*args, **kwargs):
    raise NotImplementedError("pysam.merge is not available in the stub")
