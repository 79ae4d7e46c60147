"""hadoop_bam — MI355X-native BAM read path with Hadoop-BAM's input API.

Mirrors org.seqdoop.hadoop_bam.{BAMInputFormat, BAMRecordReader, FileVirtualSplit,
SAMRecordWritable, BAMSplitGuesser, util.BGZFSplitGuesser, SplittingBAMIndex}; compute runs
in libhbam.so (HIP, gfx950) through the C ABI of include/hbam.h.
"""
from ._lib import Context, HbamUnavailable, load  # noqa: F401
from .formats import (  # noqa: F401
    AnySAMInputFormat, BAMInputFormat, BAMRecordReader, BAMSplitGuesser, BGZFSplitGuesser,
    Configuration, FileSplit, FileVirtualSplit, SAMRecordWritable, SplittingBAMIndex,
    compute_file_splits)
