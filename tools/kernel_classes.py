#!/usr/bin/env python3
"""Group a prof_summary kernel table (markdown, ms/step column) into classes.

  python tools/kernel_classes.py profiles/r02_prof19_..._kernels.md
"""
import re
import sys

CLASSES = [
    ("BatchNorm passes (bn_act.hip)", r"cml::.*bn_(apply|stats|bwd|finalize|apply2|bwd_apply2|bwd_reduce2)"),
    ("fused 1x1 conv + BN (conv1x1.hip, conv1x1g.hip)",
     r"cml::.*(conv1x1_bn|conv1x1_bnbwd|bn_bwd_coeffs|conv1x1g_|conv1x1q_)"),
    ("3x3 weight gradient (wgrad3x3.hip, wgrad DMA stride-2)",
     r"cml::.*(wgrad3x3|wgrad_dma_kernel<\d+, \d+, \d+, \d+, true)"),
    ("recompute-tail algebra (tail_prep.hip, bn_stats_gram)", r"cml::.*(tail_|bn_stats_gram)"),
    ("1x1 weight gradient (wgrad1x1.hip)", r"cml::.*(wgrad1x1|wgrad_dma_kernel|wgrad_fold)"),
    ("3x3 conv fwd + data gradient (conv_gemm.hip, gemm.hip conv mode, conv3x3p.hip)",
     r"cml::.*(conv_gemm|gemm_nt_kernel<\d, true(, \d+(, (true|false))?)?>|conv3x3p)"),
    ("own GEMM (gemm.hip: 1x1 convs as GEMMs, transformer linears)", r"cml::.*gemm_nt_kernel"),
    ("stem / pool (stem_conv.hip, pool.hip)", r"cml::.*(stem_|maxpool|bn_relu_max)"),
    ("aggregation + optimizer (agg_update, gram, weights)", r"cml::.*(agg_|gram|robust_weights|weights_kernel|fault)"),
    ("conv fwd (MIOpen / CK)", r"(grouped_conv_fwd|igemm_fwd|conv_fwd)"),
    ("conv dgrad (MIOpen / CK)", r"(igemm_bwd|grouped_conv_bwd_data)"),
    ("conv wgrad (MIOpen / CK)", r"(igemm_wrw|grouped_conv_bwd_weight)"),
    ("GEMM (hipBLASLt)", r"(Cijk_|Custom_Cijk)"),
    ("other cml kernels", r"cml::"),
]


def main(path):
    tot = {}
    total = 0.0
    for line in open(path):
        if not line.startswith("| `"):
            continue
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        name, ms = cells[0], float(cells[-1])
        total += ms
        for cls, pat in CLASSES:
            if re.search(pat, name):
                tot[cls] = tot.get(cls, 0.0) + ms
                break
        else:
            tot["other (fills, copies, elementwise)"] = tot.get("other (fills, copies, elementwise)", 0.0) + ms
    print("| class | ms / step | % |")
    print("|---|---|---|")
    for cls, ms in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"| {cls} | {ms:.2f} | {100 * ms / total:.1f} |")
    print(f"| total (listed kernels) | {total:.2f} | 100 |")


if __name__ == "__main__":
    main(sys.argv[1])
