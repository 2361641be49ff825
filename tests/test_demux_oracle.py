"""The demux oracle (oracle/demux_oracle.py) against the reference's own outputs."""
import gzip
import os

import pytest

from demux_harness import case_names, run_case


def _oracle_demux(args):
    """The oracle returns decoded output contents; write them as the reference would."""
    from oracle import demux_oracle
    outs = demux_oracle.demux(args)
    for path, data in outs.items():
        with gzip.open(path, "wb") as f:
            f.write(data)


@pytest.mark.parametrize("name", case_names())
def test_demux_oracle_matches_reference(name):
    diffs = run_case(name, _oracle_demux)
    assert not diffs, "\n".join(diffs)


def test_demux_cases_present():
    assert len(case_names()) >= 15


def _oracle_demux_files(args):
    """The timing port (bench.py --cfg5): the oracle writes the outputs itself, through gzip.open
    writers line by line as the reference does."""
    from oracle import demux_oracle
    demux_oracle.demux(args, write_files=True)


@pytest.mark.parametrize("name", case_names())
def test_demux_oracle_file_writers_match_reference(name):
    diffs = run_case(name, _oracle_demux_files)
    assert not diffs, "\n".join(diffs)
