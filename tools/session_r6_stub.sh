set -o pipefail
O=gpurun_out/stub_r6a.log
: > $O
timeout -k 10 120 python3 -u tools/rbuild_only.py --mode strict >> $O 2>&1 &&
timeout -k 10 120 python3 -u tools/rbuild_only.py --mode fast >> $O 2>&1 &&
ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_stubtx.so timeout -k 10 120 python3 -u tools/rbuild_only.py >> $O 2>&1 &&
ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_stubdiv.so timeout -k 10 120 python3 -u tools/rbuild_only.py >> $O 2>&1 &&
ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_stuball.so timeout -k 10 120 python3 -u tools/rbuild_only.py >> $O 2>&1
