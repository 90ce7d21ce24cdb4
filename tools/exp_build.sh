#!/bin/bash
# experiment variants of libg2n: tools/exp_build.sh NAME "-DFOO=1 ..." -> gfa2network_amd/_lib/exp_NAME.so
set -e
cd "$(dirname "$0")/../gfa2network_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 -I../../include $2 -c -o ../_lib/exp_$1.o g2n_pipeline.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -lz -lpthread -o ../_lib/exp_$1.so ../_lib/exp_$1.o ../_lib/g2n_host.o ../_lib/g2n_ingest.o ../_lib/g2n_pinflate.o ../_lib/g2n_split.o ../_lib/g2n_writers.o ../_lib/g2n_synth.o
rm -f ../_lib/exp_$1.o
