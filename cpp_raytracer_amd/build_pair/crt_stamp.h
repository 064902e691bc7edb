#define CRT_SOURCE_SHA "6b949073f5e809ed"
#define CRT_GIT "bbb42c361855+dirty"
