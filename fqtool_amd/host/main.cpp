// main.cpp -- `fqtool`: drop-in command line for the reference's `fqtool` (src/main.cpp) whose
// per-pack hot path runs on MI355X through libfqengine.so.
#include "processor.h"

int main(int argc, char** argv) { return fqhost::run_tool(argc, argv, true); }
