T=tools/gpu_step.sh
HCRAG_DEBUG_UNIT=1 $T u 300 python -u tests/debug/unit_dev_check.py
