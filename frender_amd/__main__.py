"""`python -m frender_amd scan|demux ...` — the reference's CLI (frender.py:817-930) on MI355X."""
import argparse
import os
import sys
from datetime import datetime, timezone


from .dist import launch_ranks


def _single_process():
    """One process, one GPU: the library loads without PyTorch (frender_amd/_runtime.py), unless something in
    this process imported it already."""
    from . import _runtime
    if "torch" not in sys.modules:
        _runtime.USE_TORCH = False


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
    p.add_argument("--gpus", type=int, default=1,
                   help="GPUs (one process each; files are sharded over them, rank 0 writes the outputs)")
    p.add_argument("files", nargs="+", help="Fastq file(s) or a directory of fastq files")
    p.set_defaults(cmd="scan")
    d = sub.add_parser("demux", help="Demultiplex paired fastq files using a frender scan result file")
    d.add_argument("-i", "--no-index-hop", action="store_true",
                   help="don't split index hop reads into their own file (will be included in undetermined file "
                        "unless -u is set)")
    d.add_argument("-a", "--no-ambiguous", action="store_true",
                   help="don't split ambiguous reads into their own file (will be included in undetermined file "
                        "unless -u is set)")
    d.add_argument("-u", "--no-undeter", action="store_true", help="do NOT produce undetermined files")
    d.add_argument("-s", "--no-samples", action="store_true", help="do NOT produce individual sample files")
    d.add_argument("-o", metavar="output_name", help="name infix for output files")
    d.add_argument("-d", metavar="output_dir",
                   default=f"./frender-demux-output_{datetime.strftime(datetime.now(timezone.utc), '%Y-%M-%d_%H%M_%Z')}/",
                   help="output directory (default: ./frender-demux-output_{date_time}/)")
    d.add_argument("-r", metavar="result_file", required=True, help="REQUIRED: frender scan result file")
    d.add_argument("--strict-header", action="store_true",
                   help="reject a results file in scan's own column order, as frender.py does (default: accept it)")
    d.add_argument("--gz-level", type=int, default=None,
                   help="gzip level of the host writers (default 9: the reference writes gzip.open's default); "
                        "the gpu writer has no levels (its streams are no larger than level 9's)")
    d.add_argument("--gz-writer", choices=("gpu", "libdeflate", "zlib"), default="gpu",
                   help="who compresses the outputs: gpu (default: the routed bytes are deflated on the GPU, "
                        "no larger than zlib level 9 makes them on FASTQ), libdeflate or zlib (host threads at "
                        "--gz-level)")
    d.add_argument("--gpus", type=int, default=1,
                   help="GPUs (one process each; file pairs are dealt to them, rank 0 writes the outputs)")
    d.add_argument("--stage-times", action="store_true", help="print the demux's seconds per stage (stderr)")
    d.add_argument("files", nargs="+", help="Fastq file, list of fastq files, or directory path")
    d.set_defaults(cmd="demux")
    args = parser.parse_args(argv)
    if getattr(args, "cmd", None) == "scan":
        if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
            return launch_ranks(args.gpus, sys.argv[1:] if argv is None else list(argv))
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            return run_rank(args)
        _single_process()
        from .scan import frender_scan
        frender_scan(args)
        return 0
    if getattr(args, "cmd", None) == "demux":
        if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
            # every rank must use the same output directory: the default names the minute
            child = (sys.argv[1:] if argv is None else list(argv))
            if "-d" not in child:
                child = child + ["-d", args.d]
            return launch_ranks(args.gpus, child)
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            return run_rank(args)
        _single_process()
        from .demux import frender_demux
        frender_demux(args)
        return 0
    parser.print_help()
    return 2


def run_rank(args) -> int:
    """One rank of a multi-GPU scan or demux (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the
    launcher or torchrun): RCCL between GPUs (FRENDER_DIST_BACKEND=gloo rehearses N ranks on fewer
    GPUs)."""
    import torch
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("FRENDER_DIST_BACKEND", "nccl")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    from .dist import PeerFailed
    try:
        if args.cmd == "demux":
            from .demux import frender_demux
            frender_demux(args)
        else:
            from .scan import frender_scan
            frender_scan(args)
    except PeerFailed:  # rank 0 raises the reference's exception; this rank just fails
        return 1
    finally:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
