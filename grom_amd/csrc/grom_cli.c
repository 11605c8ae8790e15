/* grom_cli.c -- the `grom` executable: a thin wrapper over grom_cli_main. */
#include "../../include/grom_amd.h"

int main(int argc, char **argv) { return grom_cli_main(argc, argv); }
