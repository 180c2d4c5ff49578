/* Internal helpers shared by the oracle's translation units (TEST INFRASTRUCTURE ONLY). */
#ifndef BXO_INTERNAL_H
#define BXO_INTERNAL_H

void bxo_xyxy2xywh(const double *x, double *y);
void bxo_xywh2xyxy(const double *x, double *y);
void bxo_xywh2tlwh(const double *x, double *y);
void bxo_tlwh2xyah(const double *x, double *y);
double bxo_iou_pair(const double *b1, const double *b2);
double bxo_fuse_one(double cost, double conf);

#endif
