"""python -m sctools_amd <Command> [args]  (CalculateCellMetrics, CalculateGeneMetrics,
MergeCellMetrics, MergeGeneMetrics, CreateCountMatrix, MergeCountMatrices)."""
import sys

from sctools_amd.platform import COMMANDS


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in COMMANDS:
        sys.stderr.write("usage: python -m sctools_amd {%s} [args]\n" % ",".join(COMMANDS))
        return 2
    return COMMANDS[argv[0]](argv[1:])


if __name__ == "__main__":
    sys.exit(main())
