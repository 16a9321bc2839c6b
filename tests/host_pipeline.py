"""Run the product's host stages (fslr_amd.cluster) on a fixture, like main.py:209-237."""
import numpy as np

import fixtures as fx
from fslr_amd import cluster


def host_prepare(name, bed=None):
    kw = fx.cli_options(name)
    if bed is None:
        bed = fx.input_bed(name)
    mask = set()
    if kw['cluster_mask']:
        allowed = set(bed['chrom'])
        for item in kw['cluster_mask'].split(','):
            if item in allowed or item == 'subtelomere':
                mask.add(item)
    lens = cluster.get_chromosome_lengths(fx.input_bam(name))
    bed, lens, mask, cmap = cluster.rename_chromosomes(bed, lens, mask)
    if kw['filter_false']:
        bed = cluster.delete_false(bed)
    fill = cluster.keep_fillings(bed)
    data = cluster.prepare_data(fill, mask, lens, threshold=500_000)
    return data, bed, kw
