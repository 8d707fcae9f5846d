"""Per-dispatch averages of every PMC counter for kernels named argv[1]* (rocprofv3 --pmc passes
under $MCS_PMC_DIR/pass*/), plus the derived per-wave / per-cycle ratios of pmc_summary."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary as ps  # noqa: E402

avg = ps.family_counters(sys.argv[1])
print(json.dumps({"counters": avg, "derived": ps.derived(avg)}, indent=1))
