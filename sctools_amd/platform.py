"""
Command-line entry points for the metric path -- same names, flags and return
codes as the reference's ``GenericPlatform`` metric commands
(``/root/reference/src/sctools/platform.py:225-381``; console scripts
``setup.py:42-49``):

  CalculateCellMetrics -i BAM -o STEM [-a GTF]
  CalculateGeneMetrics -i BAM -o STEM
  MergeCellMetrics FILES... -o STEM
  MergeGeneMetrics FILES... -o STEM

New flags are optional only: ``--float-mode {welford,exact}`` and ``--device``.
Run as ``python -m sctools_amd <Command> [args]``.
"""

import argparse
from typing import Iterable, Set

from sctools_amd import gtf, metrics


def _engine_args(parser):
    parser.add_argument("--float-mode", default="welford", choices=["welford", "exact"],
                        help="welford: bit-identical to sctools (default); exact: order-free exact sums")
    parser.add_argument("--device", default=None, help="torch device (default: current GPU)")


class GenericPlatform:
    @classmethod
    def calculate_gene_metrics(cls, args: Iterable[str] = None) -> int:
        parser = argparse.ArgumentParser()
        parser.add_argument("-i", "--input-bam", required=True, help="Input bam file name.")
        parser.add_argument("-o", "--output-filestem", required=True, help="Output file stem.")
        _engine_args(parser)
        args = parser.parse_args(args) if args is not None else parser.parse_args()
        g = metrics.gatherer.GatherGeneMetrics(args.input_bam, args.output_filestem,
                                               float_mode=args.float_mode, device=args.device)
        g.extract_metrics()
        return 0

    @classmethod
    def calculate_cell_metrics(cls, args: Iterable[str] = None) -> int:
        parser = argparse.ArgumentParser()
        parser.add_argument("-i", "--input-bam", required=True, help="Input bam file name.")
        parser.add_argument("-o", "--output-filestem", required=True, help="Output file stem.")
        parser.add_argument("-a", "--gtf-annotation-file", required=False, default=None,
                            help="gtf annotation file that bam_file was aligned against")
        _engine_args(parser)
        args = parser.parse_args(args) if args is not None else parser.parse_args()
        mito: Set[str] = set()
        if args.gtf_annotation_file:
            mito = gtf.get_mitochondrial_gene_names(args.gtf_annotation_file)
        g = metrics.gatherer.GatherCellMetrics(args.input_bam, args.output_filestem, mito,
                                               float_mode=args.float_mode, device=args.device)
        g.extract_metrics()
        return 0

    @classmethod
    def merge_gene_metrics(cls, args: Iterable[str] = None) -> int:
        parser = argparse.ArgumentParser()
        parser.add_argument("metric_files", nargs="+", help="Input metric files")
        parser.add_argument("-o", "--output-filestem", required=True, help="Output file stem.")
        args = parser.parse_args(args) if args is not None else parser.parse_args()
        metrics.merge.MergeGeneMetrics(args.metric_files, args.output_filestem).execute()
        return 0

    @classmethod
    def merge_cell_metrics(cls, args: Iterable[str] = None) -> int:
        parser = argparse.ArgumentParser()
        parser.add_argument("metric_files", nargs="+", help="Input metric files")
        parser.add_argument("-o", "--output-filestem", required=True, help="Output file stem.")
        args = parser.parse_args(args) if args is not None else parser.parse_args()
        metrics.merge.MergeCellMetrics(args.metric_files, args.output_filestem).execute()
        return 0


class TenXV2(GenericPlatform):
    """The reference exposes the metric commands on TenXV2 too (platform.py:579)."""


COMMANDS = {
    "CalculateCellMetrics": GenericPlatform.calculate_cell_metrics,
    "CalculateGeneMetrics": GenericPlatform.calculate_gene_metrics,
    "MergeCellMetrics": GenericPlatform.merge_cell_metrics,
    "MergeGeneMetrics": GenericPlatform.merge_gene_metrics,
}
