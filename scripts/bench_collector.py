"""The bench's f1_collector_200_connections line alone (bench.collector_config)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.collector_config(torch, torch.device("cuda", 0))))
