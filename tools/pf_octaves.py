"""Per-octave durations of the fast-pyramid kernels in gpurun_out/pf_v{0,1}
(tools/ab_fast.sh): the last step's launches, in order."""
import csv
import sys

for v in (0, 1):
    try:
        rows = list(csv.DictReader(open(f'gpurun_out/pf_v{v}/run_kernel_trace.csv')))
    except OSError:
        continue
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ks = [(r['Kernel_Name'], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, r['Grid_Size_X'],
           r['Grid_Size_Y']) for r in rows if 'pyr' in r['Kernel_Name'] or 'base9' in r['Kernel_Name']]
    n = 6 if v == 0 else 5
    print(f'SIFT_HIP_FAST_V1={v}: total {sum(k[1] for k in ks[-n:]):.1f} us')
    for k in ks[-n:]:
        print('   ', k)
