#!/bin/bash
# relink_qw.sh — fast iteration on the QW kernel: recompile score_qw.hip only and relink the
# library (make rebuilds every object on any header change).
set -e
cd "$(dirname "$0")/../hc-rag_amd/csrc"
O=../lib/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -I../../include -Wall -Wno-unused-result -Wno-unused-variable -Wno-unused-function -c score_qw.hip -o $O/score_qw.hip.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $O/hcrag_index.hip.o $O/score_qs.hip.o $O/score_qw.hip.o $O/encoder.hip.o $O/relevance.hip.o $O/multi.hip.o $O/wordpiece.cpp.o $O/errors.cpp.o -ldl -o ../lib/libhcrag_hip.so
touch $O/score_qw.hip.o
