# builds scripts/build/dropin_{old,new}: scripts/dropin_bench.c over the
# drop-in of commit $1 (old) and of the working tree (new)
set -e
cd "$(dirname "$0")"
mkdir -p build
git show "${1:-HEAD}":level-ip_amd/csrc/csum_cpu.c > build/csum_cpu_old.c
cp ../level-ip_amd/csrc/csum_cpu.c build/csum_cpu_new.c
for v in old new; do
  gcc -O2 -fPIC -Wall -shared -I../include build/csum_cpu_$v.c -o build/libdropin_$v.so
  gcc -O2 dropin_bench.c -o build/dropin_$v -Lbuild -l:libdropin_$v.so -Wl,-rpath,'$ORIGIN'
done
