"""`python -m frender_amd scan ...` — the reference's CLI (frender.py:817-930), scan on MI355X."""
import argparse
import sys


def main(argv=None):
    parser = argparse.ArgumentParser(prog="frender_amd")
    sub = parser.add_subparsers()
    p = sub.add_parser("scan", help="Scan file(s) or directory and compare to a supplied barcode table")
    p.add_argument("-n", metavar="[int]", type=int, required=True,
                   help="REQUIRED: Number of mismatches allowed between supplied barcodes and fastq file(s)")
    p.add_argument("-rc", action="store_true",
                   help="Scan/demultiplex using reverse complement of index 2 as well as forward sequence")
    p.add_argument("-c", metavar="cores", type=float, default=1,
                   help="Host cores (0 = all, (0,1) = fraction, >=1 = count); default 1")
    p.add_argument("-s", metavar="sample", type=int,
                   help="If set, sample an absolute number of reads from the head of each file (s >= 1)")
    p.add_argument("-o", metavar="output_name", help="name infix for output files")
    p.add_argument("-p", metavar="fix_prefix",
                   help="When matching sample ids to filenames, remove this prefix from the sample id")
    p.add_argument("-b", metavar="barcode_table",
                   help=".csv barcode association table; required unless a directory holding one is given")
    p.add_argument("files", nargs="+", help="Fastq file(s) or a directory of fastq files")
    p.set_defaults(cmd="scan")
    args = parser.parse_args(argv)
    if getattr(args, "cmd", None) != "scan":
        parser.print_help()
        return 2
    from .scan import frender_scan
    frender_scan(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
