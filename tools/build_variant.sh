#!/bin/bash
# Build an A/B variant of libwsg.so with extra -D flags into cppserver_amd/_build/var/<name>/.
#   tools/build_variant.sh NAME [-DFOO=1 ...]     ($KSRC / $CSRC: another wsg_kernels.hip / wsg_capi.hip, e.g. an older revision)
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/cppserver_amd/_build/var/$name
mkdir -p "$out"
cd "$out"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$root/include $*"
$H $F -I$root/cppserver_amd/csrc -c ${KSRC:-$root/cppserver_amd/csrc/wsg_kernels.hip} -o k.o
$H $F -I$root/cppserver_amd/csrc -c ${CSRC:-$root/cppserver_amd/csrc/wsg_capi.hip} -o c.o
$H -O3 -std=c++17 -fPIC -I$root/include -c $root/cppserver_amd/csrc/ws.cpp -o w.o
$H -O3 -std=c++17 -fPIC -I$root/include -c $root/cppserver_amd/csrc/ws_api.cpp -o a.o
$H -O3 -std=c++17 -fPIC -I$root/include -c $root/cppserver_amd/csrc/ws_batch.cpp -o b.o
$H -O3 -std=c++17 -fPIC -I$root/include -c $root/cppserver_amd/csrc/http.cpp -o h.o
$H -O3 -std=c++17 -fPIC -I$root/include -c $root/cppserver_amd/csrc/tls.cpp -o t.o
$H -O3 -std=c++17 -fPIC -I$root/include -c $root/cppserver_amd/csrc/wss.cpp -o s.o
$H -O3 -std=c++17 -fPIC -I$root/include -c $root/cppserver_amd/csrc/wsg_mgpu.cpp -o m.o
$H --offload-arch=gfx950 -shared -o libwsg.so k.o c.o w.o a.o b.o h.o t.o s.o m.o -lssl -lcrypto -ldl -L/opt/rocm/lib -lrocprofiler-sdk-roctx
echo "$out/libwsg.so"
