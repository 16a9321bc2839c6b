"""Golden vectors for the `.mappings.bed` producer.

Writes a synthetic BAM covering what collect_mapping_info.py branches on (multi-alignment reads
with supplementary / secondary records, reverse strands relative to the primary, soft and hard
clips, several unflagged "primaries" chosen by AS, unmapped records, one-alignment reads with a
primer-side gap <= 5 — p1 labelled, p2 labelled, both False, gaps at both ends —, extra tags), a
regions bed, and the reference's own output of ``mapping_info`` on it (with and without
regions), run through tests/golden/refharness.py (pysam stand-in decoding the records in pure
Python).  Also a BAM whose read has no primary ('flag problem' quit).

    python tests/golden/make_bam_golden.py        (needs /root/reference; writes tests/golden/bam/)
"""
import contextlib
import io
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from fslr_amd.bam import write_bam  # noqa: E402

OUT = os.path.join(HERE, 'bam')
REFS = [('chr1', 5_000_000), ('chr2', 4_000_000), ('chrX', 3_000_000), ('chr17', 2_000_000)]
PRIMERS = {'21q1': 'CTACCTCTCTCGACACCAAG', '17p6': 'GGCTGAACTATAGCCTCTGC'}


def rand_seq(rng, n):
    return ''.join(rng.choice('ACGT') for _ in range(n))


def make_records(seed=3, n_reads=400):
    rng = random.Random(seed)
    recs = []
    labels = ['21q1F', '21q1R', '17p6F', '17p6R', 'False']
    for k in range(n_reads):
        l1, l2 = rng.choice(labels), rng.choice(labels)
        name = f'r{k:05d}.{l1}_{l2}' if rng.random() < 0.9 else f'read_{k}.{l1}_{l2}'
        kind = rng.random()
        qlen = rng.randint(800, 6000)
        seq = rand_seq(rng, qlen)
        if kind < 0.22:                                   # one alignment: primer rows
            g1 = rng.choice([0, 2, 5, 6, 30])
            g2 = rng.choice([0, 3, 5, 6, 40])
            m = qlen - g1 - g2
            cig = ([('S', g1)] if g1 else []) + [('M', m)] + ([('S', g2)] if g2 else [])
            flag = rng.choice([0, 16])
            recs.append(dict(qname=name, flag=flag, tid=rng.randrange(4), pos=rng.randrange(10_000, 1_900_000),
                             mapq=rng.randrange(61), cigar=cig, seq=seq if not flag & 16 else seq,
                             tags=[('NM', 'i', rng.randrange(9)), ('AS', 'i', rng.randrange(50, 900))]))
            continue
        n_al = rng.randint(2, 7)
        lens = [rng.randint(100, 1200) for _ in range(n_al)]
        qlen = sum(lens)
        seq = rand_seq(rng, qlen)
        cuts = [sum(lens[:i]) for i in range(1, n_al)]
        segs = list(zip([0] + cuts, cuts + [qlen]))
        pri = rng.randrange(n_al)
        pri_rev = rng.random() < 0.5
        two_primaries = rng.random() < 0.1
        alt = (pri + 1) % n_al
        for j, (a, b) in enumerate(segs):
            rev = pri_rev if rng.random() < 0.6 else not pri_rev
            is_pri = j == pri or (two_primaries and j == alt)
            if is_pri:
                flag = 16 if rev else 0
                clip = 'S'
            else:
                flag = (2048 if rng.random() < 0.85 else 256) | (16 if rev else 0)
                clip = 'H' if rng.random() < 0.7 else 'S'
            left, right = (a, qlen - b) if not rev else (qlen - b, a)
            mid = b - a
            ins = rng.randrange(0, 4)
            dl = rng.randrange(0, 6)
            m1 = mid // 2
            body = [('M', m1), ('I', ins), ('M', mid - m1 - ins)] if ins else [('M', mid)]
            if dl:
                body = body[:-1] + [('D', dl)] + body[-1:] if len(body) > 1 else [('M', mid // 3), ('D', dl),
                                                                                   ('M', mid - mid // 3)]
            cig = ([(clip, left)] if left else []) + body + ([(clip, right)] if right else [])
            qlen_here = sum(n for op, n in cig if op in 'MIS=X')
            s = seq[:qlen_here] if (is_pri or clip == 'S') else seq[:qlen_here]
            tags = [('NM', 'i', rng.randrange(20)), ('AS', 'i', rng.randrange(40, 3000))]
            if rng.random() < 0.3:
                tags.insert(0, ('XA', 'Z', 'chr1,+100,50M,0;'))
            if rng.random() < 0.2:
                tags.append(('ZF', 'f', 0.5))
            recs.append(dict(qname=name, flag=flag, tid=rng.randrange(4), pos=rng.randrange(10_000, 1_900_000),
                             mapq=rng.randrange(61), cigar=cig, seq=s, tags=tags))
        if rng.random() < 0.05:                            # an unmapped record of the read
            recs.append(dict(qname=name, flag=4, tid=-1, pos=-1, mapq=0, cigar=[], seq=seq[:50], tags=[]))
    return recs


def regions_text():
    return 'chr1\t100000\t400000\nchr1\t900000\t950000\nchr2\t0\t300000\nchr17\t1500000\t1600000\n'


def main():
    import refharness
    refharness.load()
    cmi = __import__('fslr.collect_mapping_info', fromlist=['mapping_info'])
    os.makedirs(OUT, exist_ok=True)
    write_bam(os.path.join(OUT, 'input.bam'), REFS, make_records())
    with open(os.path.join(OUT, 'regions.bed'), 'w') as fh:
        fh.write(regions_text())
    cmi.mapping_info(os.path.join(OUT, 'input.bam'), os.path.join(OUT, 'expected.mappings.bed'), None, PRIMERS)
    cmi.mapping_info(os.path.join(OUT, 'input.bam'), os.path.join(OUT, 'expected_regions.mappings.bed'),
                     os.path.join(OUT, 'regions.bed'), PRIMERS)
    # a read with no unflagged record: the reference prints 'flag problem' and quits
    bad = make_records(seed=4, n_reads=20)
    bad.append(dict(qname='zz.21q1F_17p6R', flag=2048, tid=0, pos=500, mapq=5, cigar=[('H', 10), ('M', 90)],
                    seq='A' * 90, tags=[('AS', 'i', 60)]))
    write_bam(os.path.join(OUT, 'flag_problem.bam'), REFS, bad)
    out = io.StringIO()
    code = None
    with contextlib.redirect_stdout(out):
        try:
            cmi.mapping_info(os.path.join(OUT, 'flag_problem.bam'), os.path.join(OUT, 'unused.bed'), None, PRIMERS)
        except SystemExit as e:
            code = e.code
    with open(os.path.join(OUT, 'producer.json'), 'w') as fh:
        json.dump({'primers': PRIMERS, 'flag_problem_stdout': out.getvalue().replace(OUT, '{DIR}'),
                   'flag_problem_exit': code,
                   'fslr_version': '0.3.10'}, fh, indent=1)
    import gzip
    import shutil
    for f in ('expected.mappings.bed', 'expected_regions.mappings.bed'):
        with open(os.path.join(OUT, f), 'rb') as src, gzip.open(os.path.join(OUT, f + '.gz'), 'wb') as dst:
            shutil.copyfileobj(src, dst)
        os.remove(os.path.join(OUT, f))
    print('wrote', OUT)


if __name__ == '__main__':
    main()
