"""fslr_amd — MI355X-native (gfx950 HIP) implementation of fslr's interval-clustering hot path.

Drop-in for the reference's ``fslr/cluster.py`` entry points (``fslr_amd.cluster``)
and its ``fslr --skip-alignment`` CLI (``fslr_amd.main:pipeline``).  The pair
evaluation and the connected components run in ``fslr_amd/libfslr_hip.so``
(C ABI: ``include/fslr_hip.h``); there is no CPU fallback.
"""
__version__ = '0.3.10+mi355x.1'
