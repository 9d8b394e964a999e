#!/bin/bash
# Negative control of tests/test_gpu_stream_order.py: the current library
# built with -DORB_CALL_ORDER=0 (no cross-stream waits; tools/build_variant.sh noorder
# "-DORB_CALL_ORDER=0" -> lib/variants/noorder.so) is
# expected to FAIL the ordering tests (calls on two streams race on the
# handle's scratch).  Prints the pytest summary and the rc.
V=orb_slam2-chinese-annotation_amd/lib/variants/noorder.so
ORB_AMD_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_stream_order.py -q --timeout 120 --timeout-method thread 2>&1 | tail -15
echo "negative control pytest rc=${PIPESTATUS[0]} (expected non-zero: 1 = failures found)"
