#!/bin/bash
# Fused MobileNet-V2 / EfficientNet-b0 images/s and per-kernel averages (bench_d4.cnn_fused)
set -u
timeout -k 10 300 python -c "
import sys, json, torch; sys.path.insert(0, 'tools'); import bench_d4
dev = torch.device('cuda:0')
for a in ('mobilenet_v2', 'efficientnet_b0'):
    r = bench_d4.cnn_fused(a, 10, 3, 256, dev)
    print(a, round(r['images_per_s']), json.dumps({k: round(v['avg_launch_us'], 1) for k, v in r['kernels'].items()}))
"
