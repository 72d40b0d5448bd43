#ifndef POLAR_HEADER_H
#define POLAR_HEADER_H

#define _NBITS       32
#define _LOG2N       5
#define _DEPTH       6

#define PAR          4
#define LOG2_PAR     2
#define N_DIVIDED    (_NBITS / PAR) 
#define DEPTH_DIV    4

#define COUNTER      sc_uint<_DEPTH>

const sc_bv<PAR> Frozen_Bits[N_DIVIDED] = {
   //0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 1, 0, 1, 1, 1, 0, 0, 0, 1, 0, 1, 1, 1, 0, 1, 1, 1, 1, 1, 1, 1, 
     "0000", "1000", "1000", "1110", "1000", "1110", "1110", "1111"
};


#endif // POLAR_HEADER_H
