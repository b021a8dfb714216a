"""Aggregate rocprofv3 counter_collection.csv files per kernel: mean counter value per dispatch."""
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:34]
        agg[name][r['Counter_Name']].append(float(r['Counter_Value']))
keys = ['SQ_WAVE_CYCLES', 'SQ_INSTS_VALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS', 'SQ_LDS_BANK_CONFLICT', 'SQ_INSTS_VMEM_WR',
        'SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_WAIT_INST_LDS', 'SQ_WAIT_ANY', 'SQ_INSTS_VMEM_RD', 'SQ_ACTIVE_INST_VALU',
        'GRBM_GUI_ACTIVE', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_VMEM', 'SQ_ACTIVE_INST_ANY',
        'SQ_INSTS_VALU_TRANS_F32', 'SQ_BUSY_CYCLES', 'SQ_INSTS_SALU', 'SQ_INSTS_SMEM', 'SQ_ACTIVE_INST_SCA',
        'SQ_INSTS_BRANCH']
short = ['WAVECYC', 'VALU', 'MFMA', 'LDS', 'BANKCF', 'VMEMWR', 'MFMABUSY', 'WAITLDS', 'WAITANY', 'VMEMRD', 'ACTVALU',
         'GUI', 'WAITINST', 'ACTLDS', 'ACTVMEM', 'ACTANY', 'TRANS', 'BUSY', 'SALU', 'SMEM', 'ACTSCA', 'BRANCH']
print(f"{'kernel':34s} " + " ".join(f"{k:>9s}" for k in short))
for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1].get('GRBM_GUI_ACTIVE', [0]))):
    vals = []
    for k in keys:
        v = d.get(k)
        vals.append(f"{sum(v)/len(v):9.3g}" if v else f"{'-':>9s}")
    print(f"{name:34s} " + " ".join(vals))
