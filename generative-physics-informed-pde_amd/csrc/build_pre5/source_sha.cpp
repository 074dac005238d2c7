extern "C" const char* gpi_source_sha(void) { return "3a06eb447742082c8638be2ef77b9b5b8cb80033"; }
