// A python3 executable for sanitizer runs of the pybind module (tools/run_sanitizers.sh): the
// interpreter embedded in a main program linked with -fsanitize=address, so the ASan runtime is
// first in the initial library list without LD_PRELOAD, and the instrumented extension module
// (_alayalitepy + the host objects of libalaya_hip.so) is loaded into it with dlopen as usual.
#include <Python.h>

int main(int argc, char **argv) { return Py_BytesMain(argc, argv); }
