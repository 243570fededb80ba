"""Barcode geometry of the 10x v2 platform (src/sctools/platform.py:34-43), for the device
FASTQ extraction (sctools_amd.fastq).  The BAM tagging entry points around them
(Attach10xBarcodes, pysam) are outside the hot path and not rebuilt."""

from .fastq import EmbeddedBarcode


class TenXV2:
    # platform.py:36-38
    cell_barcode = EmbeddedBarcode(start=0, end=16, quality_tag='CY', sequence_tag='CR')
    molecule_barcode = EmbeddedBarcode(start=16, end=24, quality_tag='UY', sequence_tag='UR')
    sample_barcode = EmbeddedBarcode(start=0, end=8, quality_tag='SY', sequence_tag='SR')

    # platform.py:40-43
    _tags = {
        'r1': (cell_barcode, molecule_barcode),
        'i1': (sample_barcode,)
    }
