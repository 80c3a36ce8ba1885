#!/usr/bin/env python3
"""Per-dispatch stall summary of scripts/gpu_f1_stall.sh's rocprofv3 passes
(kernel trace + three --pmc passes of tools/f1_deliver_bench.py --patterns):
wave-cycle split (SQ_WAIT_ANY = parked on s_waitcnt, SQ_WAIT_INST_ANY =
issue-stalled, SQ_ACTIVE_INST_ANY), texture-addresser busy per TA instance
(TA_TA_BUSY_sum / 256 / (GRBM_GUI_ACTIVE / 8)), TCP pending stalls and the
TCC write/read requests, for every dispatch of at least 20 us.

  python tools/pmc_stall_summary.py [gpurun_out/f1stall]
"""
import sys
import csv,collections
root=sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/f1stall'
def short(k):
    if 'deliver_kernel' in k: return 'deliver<'+k.split('deliver_kernel<')[1].split('>')[0]+'>'
    if 'store_pattern' in k: return 'store_pat<'+k.split('store_pattern_kernel<')[1].split('>')[0]+'>'
    if 'segment_gather' in k: return 'gather'
    return k[:40]
seq=collections.defaultdict(list)
for r in csv.DictReader(open(f'{root}/kt/f1_kernel_trace.csv')):
    seq[short(r['Kernel_Name'])].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
data=collections.defaultdict(lambda: collections.defaultdict(float))
for p in ('p1','p2','p3'):
    per=collections.OrderedDict()
    for r in csv.DictReader(open(f'{root}/{p}/f1_counter_collection.csv')):
        key=(int(r['Dispatch_Id']),short(r['Kernel_Name']))
        per.setdefault(key,collections.defaultdict(float))[r['Counter_Name']]+=float(r['Counter_Value'])
    idx=collections.Counter()
    for (d,k),cs in sorted(per.items()):
        i=idx[k]; idx[k]+=1
        for c,v in cs.items(): data[(k,i)][c]=v
for (k,i),cs in sorted(data.items()):
    d=seq[k][i] if i < len(seq[k]) else 0
    if d < 20: continue
    g=cs.get('GRBM_GUI_ACTIVE',1)/8
    print(f"{k:28s}#{i} {d:7.1f}us waves={cs['SQ_WAVES']:.0f} vmwr={cs['SQ_INSTS_VMEM_WR']:.0f} "
          f"wait={cs['SQ_WAIT_ANY']/cs['SQ_WAVE_CYCLES']:.2f} issue={cs['SQ_WAIT_INST_ANY']/cs['SQ_WAVE_CYCLES']:.2f} act={cs['SQ_ACTIVE_INST_ANY']/cs['SQ_WAVE_CYCLES']:.2f} "
          f"TAbusy={cs['TA_TA_BUSY_sum']/256/g:.2f} TAstallTC={cs['TA_ADDR_STALLED_BY_TC_CYCLES_sum']/256/g:.2f} TCPpend={cs['TCP_PENDING_STALL_CYCLES_sum']/256/g:.2f} "
          f"wrreq={cs['TCC_EA0_WRREQ_sum']:.3g} wr64={cs['TCC_EA0_WRREQ_64B_sum']:.3g} rdreq={cs['TCC_EA0_RDREQ_sum']:.3g} wrstall={cs['TCC_EA0_WRREQ_STALL_sum']:.3g}")
