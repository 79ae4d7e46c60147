"""hadoop_bam — MI355X-native BAM read path with Hadoop-BAM's input API.

Mirrors org.seqdoop.hadoop_bam.{BAMInputFormat, BAMRecordReader, FileVirtualSplit,
SAMRecordWritable, BAMSplitGuesser, util.BGZFSplitGuesser, util.BGZFBlockIndexer/BGZFBlockIndex/BGZFSplitFileInputFormat, SplittingBAMIndex, SplittingBAMIndexer}, the Sort plugin's
shuffle sort (cli/plugins/Sort) and its BAM output (BAMRecordWriter, KeyIgnoringBAMOutputFormat,
util.SAMOutputPreparer, cli.Utils.mergeSAMInto); compute runs
in libhbam.so (HIP, gfx950) through the C ABI of include/hbam.h.
"""
from ._lib import Context, HbamUnavailable, load  # noqa: F401
from .formats import (  # noqa: F401
    AnySAMInputFormat, BAMInputFormat, BGZFBlockIndex, BGZFBlockIndexer, BGZFSplitFileInputFormat, BAMRecordReader, BAMSplitGuesser, BGZFSplitGuesser,
    Configuration, FileSplit, FileVirtualSplit, SAMRecordWritable, SplittingBAMIndex,
    SplittingBAMIndexer, compute_file_splits)
from .sort import HipSortOps, RcclComm, SortedRun, sort_sharded  # noqa: F401
from .output import (  # noqa: F401
    BAMRecordWriter, KeyIgnoringBAMOutputFormat, KeyIgnoringBAMRecordWriter, SAMFileHeader,
    SAMOutputPreparer, merge_sam_into, read_sam_header)
